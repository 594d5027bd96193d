// Round-level prover session (interactive.cpp): the reference's ProverFirstState ..
// ProverSecondSumcheckState (/root/reference/src/ahp/prover.rs:24-64) behind one handle.
#pragma once
#include <deque>
#include <exception>
#include <memory>
#include <thread>
#include <vector>

#include "prover.hpp"

namespace spx {

struct Interactive {
    enum { kFirst = 1, kSecond, kThird, kSumcheck1, kFourth, kFifth, kSumcheck2, kDone };
    Ctx& C;
    Index& I;
    std::unique_ptr<Witness> W;
    PP* pp = nullptr;
    int next = kFirst;  // the step the caller may take now
    int rounds = 0;     // sumcheck rounds taken in the current sumcheck

    Interactive(Ctx& c, Index& i, std::unique_ptr<Witness> w);
    ~Interactive();  // a session freed mid-way cancels its worker at the next coin it waits for

    std::vector<uint8_t> first_round(PP* P);
    std::vector<uint8_t> second_round(const uint8_t* r_v, size_t n, PP* P);
    std::vector<uint8_t> third_round(const uint8_t* tau, size_t n);
    std::vector<uint8_t> sumcheck_round(int which, const uint8_t* challenge_or_null);
    std::vector<uint8_t> fourth_round(const uint8_t* last_point);
    std::vector<uint8_t> fifth_round(const uint8_t* rabc);
    std::vector<uint8_t> sixth_round(const uint8_t* last_point, PP* P);

   private:
    struct Coins;
    void start(PP* P);
    std::vector<uint8_t> step(int expect, const std::vector<host::Fr>& give, size_t want_msgs);
    std::mutex mu;
    std::condition_variable cv;
    std::deque<host::Fr> coins;
    std::vector<std::vector<uint8_t>> msgs;
    size_t taken = 0;
    bool cancel = false, finished = false;
    std::exception_ptr err;
    std::vector<uint8_t> final_proof;
    std::unique_ptr<Coins> coins_;
    std::thread th;
    CtxClaim claim;  // held from construction until the worker's prove() returns
};

}  // namespace spx
