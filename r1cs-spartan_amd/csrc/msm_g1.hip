// G1 instantiation of the MSM / PP-preprocessing / keygen kernels (see msm_impl.hpp).
#include "msm_impl.hpp"

namespace spx {

void msm_run_g1(MsmWorkspace* ws, const MsmInst* insts, int ninst, const G1Slot* pts, const Fr* scalars, void* out,
                hipStream_t s, const MsmShard& sh) {
    msm_run_t<Fq>(ws, insts, ninst, pts, scalars, out, s, sh);
}
void precompute_windows_g1(const G1Aff* raw, uint64_t count, bool pair_sum, int c, int W, G1Aff* dst, void* tmp,
                           hipStream_t s) {
    precompute_windows_t<Fq>(raw, count, pair_sum, c, W, dst, tmp, s);
}
void fixed_base_g1(const G1Aff* table, const Fr* scalars, uint64_t n, G1Aff* out, void* tmp, hipStream_t s) {
    fixed_base_t<Fq>(table, scalars, n, out, tmp, s);
}

}  // namespace spx
