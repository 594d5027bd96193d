// RCCL communicator: one process per GPU, torch.distributed (or any out-of-band channel)
// distributes the ncclUniqueId. Only tiny messages cross it (3 Fr per sumcheck round, one affine
// point per MSM and rank), so a latency-bound AllGather over xGMI is all the prover needs.
#include <rccl/rccl.h>

#include "prover.hpp"

namespace spx {

#define SPX_NCCL(x)                                                                                     \
    do {                                                                                                \
        ncclResult_t r_ = (x);                                                                          \
        if (r_ != ncclSuccess) throw SpxError(kDevice, std::string("RCCL: ") + ncclGetErrorString(r_)); \
    } while (0)

struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    int r, w;
    hipStream_t s;
    DevMem sbuf, rbuf;
    RcclComm(const uint8_t id[128], int rank, int world, hipStream_t st) : r(rank), w(world), s(st) {
        ncclUniqueId uid;
        static_assert(sizeof(uid) == 128, "ncclUniqueId size");
        memcpy(&uid, id, 128);
        SPX_NCCL(ncclCommInitRank(&comm, world, uid, rank));
    }
    ~RcclComm() override {
        if (comm) ncclCommDestroy(comm);
    }
    int rank() const override { return r; }
    int size() const override { return w; }
    void allgather(const void* send, void* recv, size_t bytes) override {
        sbuf.ensure(bytes);
        rbuf.ensure(bytes * w);
        SPX_HIP(hipMemcpyAsync(sbuf.p, send, bytes, hipMemcpyHostToDevice, s));
        SPX_NCCL(ncclAllGather(sbuf.p, rbuf.p, bytes, ncclUint8, comm, s));
        SPX_HIP(hipMemcpyAsync(recv, rbuf.p, bytes * w, hipMemcpyDeviceToHost, s));
        SPX_HIP(hipStreamSynchronize(s));
    }
};

std::unique_ptr<Comm> make_rccl_comm(const uint8_t id[128], int rank, int world, int device, hipStream_t s) {
    SPX_HIP(hipSetDevice(device));
    return std::unique_ptr<Comm>(new RcclComm(id, rank, world, s));
}

}  // namespace spx

extern "C" int spx_comm_unique_id_impl(uint8_t out[128]) {
    ncclUniqueId uid;
    if (ncclGetUniqueId(&uid) != ncclSuccess) return 5;
    memcpy(out, &uid, 128);
    return 0;
}
