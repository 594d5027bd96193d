// RCCL communicator: one process per GPU, torch.distributed (or any out-of-band channel)
// distributes the ncclUniqueId. Only tiny messages cross it (3 Fr per sumcheck round, one affine
// point per MSM and rank), so a latency-bound AllGather over xGMI is all the prover needs.
#include <rccl/rccl.h>

#include <algorithm>

#include "prover.hpp"

namespace spx {

#define SPX_NCCL(x)                                                                                     \
    do {                                                                                                \
        ncclResult_t r_ = (x);                                                                          \
        if (r_ != ncclSuccess) throw SpxError(kDevice, std::string("RCCL: ") + ncclGetErrorString(r_)); \
    } while (0)

// The exchange runs on the communicator's OWN stream, with pinned staging: the host waits only for
// the collective, never for the proof's queued kernels (the commitment MSM keeps running while the
// transcript state is exchanged). Several proofs in flight share ONE communicator through the
// ordered exchange hub (comm_hub.cpp): independent communicators driven by independent threads
// could order their collectives differently on different ranks.
struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    int r, w, dev;
    hipStream_t s = nullptr;
    DevMem sbuf, rbuf;
    uint8_t *hs = nullptr, *hr = nullptr;
    size_t hcap = 0;
    RcclComm(const uint8_t id[128], int rank, int world, int device) : r(rank), w(world), dev(device) {
        ncclUniqueId uid;
        static_assert(sizeof(uid) == 128, "ncclUniqueId size");
        memcpy(&uid, id, 128);
        SPX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        SPX_NCCL(ncclCommInitRank(&comm, world, uid, rank));
    }
    ~RcclComm() override {
        if (comm) ncclCommDestroy(comm);
        if (hs) (void)hipHostFree(hs);
        if (hr) (void)hipHostFree(hr);
        if (s) (void)hipStreamDestroy(s);
    }
    int rank() const override { return r; }
    int size() const override { return w; }
    void allgather(const void* send, void* recv, size_t bytes) override {
        SPX_HIP(hipSetDevice(dev));  // the calling thread may be an exchange hub's (device 0 by default)
        if (bytes * w > hcap) {  // grow only between calls: the previous call synchronised s
            if (hs) SPX_HIP(hipHostFree(hs));
            if (hr) SPX_HIP(hipHostFree(hr));
            hs = hr = nullptr;
            hcap = std::max<size_t>(bytes * w, 4096);
            SPX_HIP(hipHostMalloc((void**)&hs, hcap));
            SPX_HIP(hipHostMalloc((void**)&hr, hcap));
        }
        sbuf.ensure(bytes);
        rbuf.ensure(bytes * w);
        memcpy(hs, send, bytes);
        SPX_HIP(hipMemcpyAsync(sbuf.p, hs, bytes, hipMemcpyHostToDevice, s));
        SPX_NCCL(ncclAllGather(sbuf.p, rbuf.p, bytes, ncclUint8, comm, s));
        SPX_HIP(hipMemcpyAsync(hr, rbuf.p, bytes * w, hipMemcpyDeviceToHost, s));
        SPX_HIP(hipStreamSynchronize(s));
        memcpy(recv, hr, bytes * w);
    }
};

std::unique_ptr<Comm> make_rccl_comm(const uint8_t id[128], int rank, int world, int device, hipStream_t) {
    SPX_HIP(hipSetDevice(device));
    return std::unique_ptr<Comm>(new RcclComm(id, rank, world, device));
}

}  // namespace spx

extern "C" int spx_comm_unique_id_impl(uint8_t out[128]) {
    ncclUniqueId uid;
    if (ncclGetUniqueId(&uid) != ncclSuccess) return 5;
    memcpy(out, &uid, 128);
    return 0;
}
