// On-node shared-memory communicator (one process per GPU, all ranks on one host).
//
// What a sharded proof exchanges is tiny and lives on the host (3 Fr per sumcheck round, a few
// affine points per MSM), because the host derives every Fiat-Shamir challenge. A
// host transport keeps those exchanges off the GPU queues entirely: with several proofs in flight
// per rank (one communicator each), device collectives issued from independent worker threads can
// reach a hardware queue (GPU_MAX_HW_QUEUES = 4) in different orders on different ranks and
// deadlock; a host allgather cannot. Latency is a few microseconds.
//
// Segment: [seq[r] (one cache line per rank)][2 buffers x world x kSlot bytes]. allgather #n writes
// this rank's slot of buffer n&1, publishes seq[r] = n (release), wakes futex waiters on it, and
// waits for every seq >= n (acquire): a short spin, then a futex sleep on the peer's counter
// (shared-mapping futexes work across processes), so hundreds of waiting proof threads on a node
// do not steal cores from the ones hashing. Buffer n&1 is rewritten only by call n+2, which every
// rank starts after finishing call n+1, i.e. after it has read call n's data.
#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/spartan_hip.h"
#include "prover.hpp"

namespace spx {

namespace {
constexpr int kMaxRanks = 64;
constexpr size_t kSlot = 1 << 16;
constexpr size_t kEpoch = 64 * kMaxRanks;  // one line after the counters: rank 0's per-run epoch
constexpr size_t kHdr = kEpoch + 64;
}  // namespace

struct ShmComm : Comm {
    int r, w;
    std::string name;
    uint8_t* base = nullptr;
    size_t len = 0;
    uint64_t n = 0;
    ShmComm(const std::string& nm, int rank, int world) : r(rank), w(world) {
        if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) invalid("shm comm: bad rank/world");
        name = "/" + nm;
        if (nm.find('/') != std::string::npos) invalid("shm comm: name must not contain '/'");
        len = kHdr + 2 * (size_t)world * kSlot;
        // rank 0 creates the segment (O_EXCL: a leftover segment of that name is an error, never
        // silently reused with stale counters) and sizes it, which zero-fills it; the others open
        // the existing object only, waiting until it exists at its full size
        int fd = -1;
        if (r == 0) {
            fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd < 0) throw SpxError(kDevice, "shm_open(O_EXCL) failed for " + name + " (name in use?)");
            if (ftruncate(fd, (off_t)len) != 0) {
                close(fd);
                shm_unlink(name.c_str());
                throw SpxError(kDevice, "ftruncate failed for " + name);
            }
        } else {
            auto t0 = std::chrono::steady_clock::now();
            for (;;) {
                fd = shm_open(name.c_str(), O_RDWR, 0600);
                if (fd >= 0) {
                    struct stat st;
                    if (fstat(fd, &st) == 0 && (size_t)st.st_size == len) break;
                    close(fd);
                    fd = -1;
                }
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600))
                    throw SpxError(kDevice, "shm comm: segment " + name + " not created by rank 0 in 600 s");
                usleep(1000);
            }
        }
        void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw SpxError(kDevice, "mmap failed for " + name);
        base = (uint8_t*)p;
        // Rank 0 stamps a per-run epoch into the fresh (zero-filled) segment; the others wait for it.
        // A segment left behind by a crashed run is refused: its counters are past the rendezvous,
        // or its epoch is not the one the live rank 0 wrote (checked after the rendezvous).
        auto& epoch = *reinterpret_cast<std::atomic<uint64_t>*>(base + kEpoch);
        if (r == 0) {
            uint64_t e = 0;
            while (!e) e = ((uint64_t)getpid() << 32) ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
            epoch.store(e, std::memory_order_release);
        } else {
            auto t0 = std::chrono::steady_clock::now();
            while (!epoch.load(std::memory_order_acquire)) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600))
                    throw SpxError(kDevice, "shm comm: segment " + name + " never initialised by rank 0");
                usleep(100);
            }
            for (int k = 0; k < world; ++k)
                if (!reached(1, seq(k).load(std::memory_order_acquire)))
                    throw SpxError(kDevice, "shm comm: segment " + name + " is in use by another run (stale name?)");
        }
        const uint64_t mine = epoch.load(std::memory_order_acquire);
        // rendezvous: every rank has mapped the segment once this completes; then drop the name
        struct Hello {
            int rank;
            int pad;
            uint64_t epoch;
        } hello{r, 0, mine};
        std::vector<Hello> all(world);
        allgather(&hello, all.data(), sizeof(Hello));
        for (int k = 0; k < world; ++k)
            if (all[k].rank != k || all[k].epoch != all[0].epoch)
                throw SpxError(kDevice, "shm comm: rank / epoch mismatch (stale segment name?)");
        if (r == 0) shm_unlink(name.c_str());
    }
    ~ShmComm() override {
        if (base) munmap(base, len);
    }
    // 32-bit counters (futex words); wrap-safe comparison
    std::atomic<uint32_t>& seq(int k) { return *reinterpret_cast<std::atomic<uint32_t>*>(base + 64 * k); }
    static bool reached(uint32_t v, uint32_t c) { return (int32_t)(v - c) >= 0; }
    static void futex_wait(std::atomic<uint32_t>* a, uint32_t expect) {
        struct timespec ts = {0, 2000000};  // 2 ms cap: re-check (and the 600 s deadline) periodically
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAIT, expect, &ts, nullptr, 0);
    }
    static void futex_wake(std::atomic<uint32_t>* a) {
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
    }
    uint8_t* slot(uint32_t call, int k) { return base + kHdr + ((call & 1) * w + k) * kSlot; }
    int rank() const override { return r; }
    int size() const override { return w; }
    void one(const uint8_t* send, uint8_t* recv, size_t bytes, size_t rstride) {
        const uint32_t c = (uint32_t)++n;
        memcpy(slot(c, r), send, bytes);
        seq(r).store(c, std::memory_order_release);
        futex_wake(&seq(r));
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < w; ++k) {
            unsigned spins = 0;
            for (;;) {
                const uint32_t v = seq(k).load(std::memory_order_acquire);
                if (reached(v, c)) break;
                if (++spins < 2048) {
                    __builtin_ia32_pause();
                    continue;
                }
                futex_wait(&seq(k), v);
                if ((spins & 0xff) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600))
                    throw SpxError(kDevice, "shm allgather: rank " + std::to_string(k) + " did not arrive in 600 s");
            }
        }
        for (int k = 0; k < w; ++k) memcpy(recv + k * rstride, slot(c, k), bytes);
    }
    void allgather(const void* send, void* recv, size_t bytes) override {
        // messages larger than a slot go in slot-sized rounds
        const uint8_t* s = (const uint8_t*)send;
        uint8_t* d = (uint8_t*)recv;
        size_t done = 0;
        do {
            size_t b = std::min(kSlot, bytes - done);
            one(s + done, d + done, b, bytes);
            done += b;
        } while (done < bytes);
    }
};

std::unique_ptr<Comm> make_shm_comm(const char* name, int rank, int world) {
    if (!name || !*name) invalid("shm comm: empty name");
    return std::unique_ptr<Comm>(new ShmComm(name, rank, world));
}

}  // namespace spx
