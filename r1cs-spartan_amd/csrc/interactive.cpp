// Interactive (round-level) prover: the reference's prover_init .. prove_sixth_round
// (/root/reference/src/ahp/prover.rs:109-281), driven round by round with verifier coins supplied by
// the caller, as ahp/tests.rs:8-70 drives it. The session runs the one product prove() (the same
// kernels, layouts and exchanges as spx_prove) on a worker thread whose transcript is external: each
// prover message is handed to the caller, and each challenge waits for the caller's next verifier
// message. So every round-level message is, byte for byte, the message the whole-proof path emits
// for the same challenges.
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

#include "interactive.hpp"

namespace spx {

namespace {
struct Cancelled {};  // unwinds a worker blocked on a coin when the session is freed
}  // namespace

struct Interactive::Coins : ExternalCoins {
    Interactive& s;
    explicit Coins(Interactive& x) : s(x) {}
    void message(const void* d, size_t n) override {
        std::lock_guard<std::mutex> lk(s.mu);
        s.msgs.emplace_back((const uint8_t*)d, (const uint8_t*)d + n);
        s.cv.notify_all();
    }
    host::Fr draw() override {
        std::unique_lock<std::mutex> lk(s.mu);
        s.cv.wait(lk, [&] { return s.cancel || !s.coins.empty(); });
        if (s.cancel) throw Cancelled{};
        host::Fr r = s.coins.front();
        s.coins.pop_front();
        return r;
    }
};

// The session claims its context from prover_init until its worker's prove() has returned (or the
// session is freed): a prove, verify or second session on the same context is refused meanwhile.
Interactive::Interactive(Ctx& c, Index& i, std::unique_ptr<Witness> w) : C(c), I(i), W(std::move(w)) { claim.take(C); }

Interactive::~Interactive() {
    {
        std::lock_guard<std::mutex> lk(mu);
        cancel = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();  // the unwinding prove drained both streams (UnwindDrain)
    claim.release();
}

void Interactive::start(PP* P) {
    pp = P;
    coins_ = std::make_unique<Coins>(*this);
    const int dev = C.device;
    th = std::thread([this, dev] {
        std::exception_ptr e;
        std::vector<uint8_t> proof;
        try {
            SPX_HIP(hipSetDevice(dev));
            ProveOpts o;
            o.coins = coins_.get();
            o.claimed = true;
            proof = prove(C, I, *W, pp, o);
        } catch (const Cancelled&) {
        } catch (...) {
            e = std::current_exception();
        }
        std::lock_guard<std::mutex> lk(mu);
        claim.release();  // prove() has returned: its streams are idle
        err = e;
        final_proof = std::move(proof);
        finished = true;
        cv.notify_all();
    });
}

std::vector<uint8_t> Interactive::step(int expect, const std::vector<host::Fr>& give, size_t want_msgs) {
    if (expect != next) invalid("round-level prover called out of order (expected step " + std::to_string(next) + ")");
    std::unique_lock<std::mutex> lk(mu);
    for (auto& c : give) coins.push_back(c);
    cv.notify_all();
    const size_t target = taken + want_msgs;
    cv.wait(lk, [&] { return finished || msgs.size() >= target; });
    if (msgs.size() < target) {
        if (err) std::rethrow_exception(err);
        throw SpxError(kDevice, "interactive prover ended early");
    }
    std::vector<uint8_t> out;
    for (; taken < target; ++taken) out.insert(out.end(), msgs[taken].begin(), msgs[taken].end());
    return out;
}

static std::vector<host::Fr> coins_of(const uint8_t* b, size_t n) {
    std::vector<host::Fr> v(n);
    for (size_t i = 0; i < n; ++i) {
        uint64_t c[4];
        memcpy(c, b + 32 * i, 32);
        if (host::Fr::geq_p(c)) throw SpxError(kSerialization, "non-canonical field element in a verifier message");
        v[i] = host::Fr::from_canon(c);
    }
    return v;
}

// prover_first_round (prover.rs:123-141): z = v || w, the commitment
std::vector<uint8_t> Interactive::first_round(PP* P) {
    if (next != kFirst) invalid("round-level prover called out of order (prover_first_round)");
    if (!P) invalid("null public parameter");
    start(P);
    auto m = step(kFirst, {}, 1);
    next = kSecond;
    return m;
}
// prover_second_round (prover.rs:143-160): r_v (log_v coins), z(r_v, 0...0) and its opening
std::vector<uint8_t> Interactive::second_round(const uint8_t* r_v, size_t n, PP* P) {
    if (P != pp) invalid("prover_second_round: a different public parameter than prover_first_round's");
    if (n != (size_t)ilog2(W->v.size() / 32)) invalid("r_v must have log2 |v| elements");
    auto m = step(kSecond, coins_of(r_v, n), 1);
    next = kThird;
    return m;
}
// prover_third_round (prover.rs:163-196): tau (log_n coins) -> IndexInfo of the first sumcheck
std::vector<uint8_t> Interactive::third_round(const uint8_t* tau, size_t n) {
    if (n != (size_t)I.log_n) invalid("tau must have log_n elements");
    auto m = step(kThird, coins_of(tau, n), 1);
    next = kSumcheck1;
    rounds = 0;
    return m;
}
// prove_first_sumcheck_round / prove_second_sumcheck_round (prover.rs:199-207, 258-266): the first
// call takes no verifier message, every later one the previous round's challenge
std::vector<uint8_t> Interactive::sumcheck_round(int which, const uint8_t* ch) {
    if (next != which) invalid("round-level prover called out of order (sumcheck round)");
    if (rounds == 0 && ch) throw SpxError(kSumcheck, "first round should be prover first");
    if (rounds > 0 && !ch) throw SpxError(kSumcheck, "verifier message is empty");
    if (rounds >= I.log_n) throw SpxError(kSumcheck, "prover is not active");
    auto m = step(which, ch ? coins_of(ch, 1) : std::vector<host::Fr>{}, 1);
    ++rounds;
    return m;
}
// prove_fourth_round (prover.rs:210-228): the last point of r_x -> va, vb, vc
std::vector<uint8_t> Interactive::fourth_round(const uint8_t* last) {
    if (next != kSumcheck1 || rounds != I.log_n) invalid("prove_fourth_round before the first sumcheck's last round");
    auto c = coins_of(last, 1);  // a non-canonical coin leaves the session where it was (retry allowed)
    next = kFourth;
    auto m = step(kFourth, c, 1);
    next = kFifth;
    return m;
}
// prove_fifth_round (prover.rs:230-255): r_a, r_b, r_c -> IndexInfo of the second sumcheck
std::vector<uint8_t> Interactive::fifth_round(const uint8_t* rabc) {
    auto m = step(kFifth, coins_of(rabc, 3), 1);
    next = kSumcheck2;
    rounds = 0;
    return m;
}
// prove_sixth_round (prover.rs:268-281): the last point of r_y -> z(r_y) and its opening proof
std::vector<uint8_t> Interactive::sixth_round(const uint8_t* last, PP* P) {
    if (next != kSumcheck2 || rounds != I.log_n) invalid("prove_sixth_round before the second sumcheck's last round");
    if (P != pp) invalid("prove_sixth_round: a different public parameter than prover_first_round's");
    {
        std::lock_guard<std::mutex> lk(mu);
        for (auto& c : coins_of(last, 1)) coins.push_back(c);
    }
    cv.notify_all();
    th.join();
    next = kDone;
    if (err) std::rethrow_exception(err);
    // the final message is the proof's tail after every fed message (ProverSixthMessage)
    size_t fed = 0;
    for (auto& m : msgs) fed += m.size();
    // proof = messages in order, with the two sumchecks' Vec length prefixes (8 bytes each) between them
    const size_t head = fed + 16;
    if (final_proof.size() < head) throw SpxError(kDevice, "interactive proof shorter than its messages");
    return std::vector<uint8_t>(final_proof.begin() + head, final_proof.end());
}

}  // namespace spx
