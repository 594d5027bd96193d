// Ordered exchange hub: ONE collective transport per process (an RCCL communicator, or the
// in-process group of the tests) shared by every proof in flight on this rank.
//
// Each context takes a channel; a proof's exchanges are a fixed sequence on its channel, the same
// on every rank (context j proves the same witnesses everywhere, spx_prove_many). Independent host
// threads reach their exchanges in different orders on different ranks, so they cannot each issue
// collectives of their own: two ranks could then wait in different collectives, and device
// collectives that wait on each other in different orders deadlock. The hub's thread alone talks
// to the transport, in rounds every rank runs identically:
//   1. control: allgather of the per-channel size of the locally pending request (0 = none);
//   2. data (only if some channel is pending on every rank): ONE allgather carrying those
//      channels' payloads, packed in channel order.
// Every rank derives the same matched set from round 1, so both ranks' transports always see the
// same collective sequence. A hub runs a round only while it has a pending request of its own; a
// request pending on one rank is matched by the same (channel, sequence) request of every other
// rank, so no rank waits in a round its peers never reach.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>

#include "prover.hpp"

namespace spx {

struct OrderedHub {
    static constexpr int kChannels = 64;
    struct Req {
        const void* send;
        void* recv;
        size_t bytes;
        bool done = false;
        std::exception_ptr err;
    };
    std::unique_ptr<Comm> base;
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    Req* pend[kChannels] = {};
    bool taken[kChannels] = {};
    bool stop = false;
    std::exception_ptr broken;  // a transport failure fails every later request too
    uint64_t st_rounds = 0, st_data = 0, st_served = 0, st_max_batch = 0, st_idle = 0;
    uint64_t arrivals = 0;  // requests posted so far (a new one ends the back-off after an idle round)
    // after a round that matched nothing, the hub waits this long (or for a new local request) before
    // the next: peers reach their side of a pending exchange later, and an immediate next round would
    // spin collectives (on RCCL a kernel plus a stream sync each) at full rate meanwhile
    static constexpr auto kIdleBackoff = std::chrono::microseconds(50);
    std::vector<uint8_t> sbuf, rbuf;
    std::thread th;

    explicit OrderedHub(std::unique_ptr<Comm> b) : base(std::move(b)) { th = std::thread([this] { run(); }); }
    ~OrderedHub() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv_work.notify_all();
        th.join();
    }
    int rank() const { return base->rank(); }
    int size() const { return base->size(); }

    void attach(int ch) {
        std::lock_guard<std::mutex> lk(mu);
        if (ch < 0 || ch >= kChannels) invalid("hub channel out of range (0..63)");
        if (taken[ch]) invalid("hub channel already attached");
        taken[ch] = true;
    }
    void detach(int ch) {
        std::lock_guard<std::mutex> lk(mu);
        taken[ch] = false;
    }

    void allgather(int ch, const void* send, void* recv, size_t bytes) {
        if (bytes >= 0xFFFFFFFFull) invalid("hub exchange larger than 4 GiB");
        Req q{send, recv, bytes};
        std::unique_lock<std::mutex> lk(mu);
        if (broken) std::rethrow_exception(broken);
        if (pend[ch]) invalid("two exchanges at once on one hub channel");
        pend[ch] = &q;
        ++arrivals;
        cv_work.notify_one();
        cv_done.wait(lk, [&] { return q.done; });
        if (q.err) std::rethrow_exception(q.err);
    }

    void fail_all(std::exception_ptr e) {  // with mu held
        broken = e;
        for (auto& p : pend)
            if (p) {
                p->err = e;
                p->done = true;
                p = nullptr;
            }
        cv_done.notify_all();
    }

    void run() {
        const int w = size();
        std::vector<uint32_t> ctl(kChannels), all((size_t)kChannels * w);
        bool idle = false;       // the previous round matched nothing
        uint64_t seen_arr = 0;   // arrivals at the previous round's snapshot
        for (;;) {
            Req* snap[kChannels];
            {
                std::unique_lock<std::mutex> lk(mu);
                auto any = [&] {
                    for (auto* p : pend)
                        if (p) return true;
                    return false;
                };
                if (idle) cv_work.wait_for(lk, kIdleBackoff, [&] { return stop || arrivals != seen_arr; });
                cv_work.wait(lk, [&] { return stop || any(); });
                if (!any()) return;  // stop, nothing pending (peers have no request this rank lacks)
                std::copy(pend, pend + kChannels, snap);
                seen_arr = arrivals;
            }
            try {
                for (int c = 0; c < kChannels; ++c) ctl[c] = snap[c] ? (uint32_t)(snap[c]->bytes + 1) : 0;
                base->allgather(ctl.data(), all.data(), sizeof(uint32_t) * kChannels);
                ++st_rounds;
                // matched channels: pending on every rank. A size disagreement is a protocol error
                // every rank sees alike: the channel fails everywhere, no data round involves it.
                size_t off[kChannels + 1], tot = 0;
                bool match[kChannels], bad[kChannels];
                int nm = 0;
                for (int c = 0; c < kChannels; ++c) {
                    bool m = true, b = false;
                    for (int k = 0; k < w; ++k) {
                        uint32_t v = all[(size_t)k * kChannels + c];
                        m = m && v != 0;
                        b = b || v != all[c];
                    }
                    match[c] = m && !b;
                    bad[c] = m && b;
                    off[c] = tot;
                    if (match[c]) {
                        tot += all[c] - 1;
                        ++nm;
                    }
                }
                off[kChannels] = tot;
                if (nm && tot) {
                    sbuf.resize(tot);
                    rbuf.resize(tot * w);
                    for (int c = 0; c < kChannels; ++c)
                        if (match[c] && snap[c]->bytes) memcpy(sbuf.data() + off[c], snap[c]->send, snap[c]->bytes);
                    base->allgather(sbuf.data(), rbuf.data(), tot);
                    ++st_data;
                    for (int c = 0; c < kChannels; ++c)
                        if (match[c])
                            for (int k = 0; k < w; ++k)
                                memcpy((uint8_t*)snap[c]->recv + (size_t)k * snap[c]->bytes,
                                       rbuf.data() + (size_t)k * tot + off[c], snap[c]->bytes);
                }
                std::lock_guard<std::mutex> lk(mu);
                for (int c = 0; c < kChannels; ++c) {
                    if (!match[c] && !bad[c]) continue;
                    if (bad[c])
                        snap[c]->err = std::make_exception_ptr(
                            SpxError(kInvalidArgument, "hub: ranks disagree on an exchange's size (channel " +
                                                           std::to_string(c) + ")"));
                    snap[c]->done = true;
                    pend[c] = nullptr;
                }
                st_served += nm;
                st_max_batch = std::max<uint64_t>(st_max_batch, nm);
                idle = nm == 0;
                st_idle += idle;
                cv_done.notify_all();
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu);
                fail_all(std::current_exception());
                return;
            }
        }
    }
};

// one context's view of the hub: a Comm whose allgathers go through channel `ch`
struct HubChannel : Comm {
    std::shared_ptr<OrderedHub> hub;
    int ch;
    HubChannel(std::shared_ptr<OrderedHub> h, int c) : hub(std::move(h)), ch(c) { hub->attach(ch); }
    ~HubChannel() override { hub->detach(ch); }
    int rank() const override { return hub->rank(); }
    int size() const override { return hub->size(); }
    void allgather(const void* s, void* r, size_t b) override {
        hub->allgather(ch, s, r, b);
    }
};

std::shared_ptr<OrderedHub> make_hub(std::unique_ptr<Comm> base) { return std::make_shared<OrderedHub>(std::move(base)); }
std::unique_ptr<Comm> make_hub_channel(const std::shared_ptr<OrderedHub>& hub, int channel) {
    return std::unique_ptr<Comm>(new HubChannel(hub, channel));
}
void hub_allgather(OrderedHub& hub, int channel, const void* send, void* recv, size_t bytes) {
    if (channel < 0 || channel >= OrderedHub::kChannels) invalid("hub channel out of range (0..63)");
    hub.allgather(channel, send, recv, bytes);
}
void hub_stats(OrderedHub& hub, uint64_t out[5]) {
    std::lock_guard<std::mutex> lk(hub.mu);
    out[0] = hub.st_rounds;
    out[1] = hub.st_data;
    out[2] = hub.st_served;
    out[3] = hub.st_max_batch;
    out[4] = hub.st_idle;
}

}  // namespace spx
