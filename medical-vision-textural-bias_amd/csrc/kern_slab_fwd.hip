// Pass A: k_slab_fwd -- per (bc, h) slab: real rows -> pair-packed R2C along D -> C2C along W.
// Compiled once per radix set (-DTB_RS).  Body: pass_a_body (fft_core.h).
#include "kernels.h"

namespace tb {
namespace {
template <int NT, int RS>
__global__ __launch_bounds__(NT) void k_slab_fwd(SlabFwdArgs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SlabFwdArgs& a = kargs<SlabFwdArgs>();
  DevCtx ctx{(int)threadIdx.x, NT};
  pass_a_body<DevCtx, RS>(ctx, reinterpret_cast<cf*>(smem), a.pl, a.x, a.sbc, a.sh, a.sw, a.S,
                          a.bc0 + (int)blockIdx.y, (int)blockIdx.x);
}
}  // namespace

template <int RS>
hipError_t launch_slab_fwd(const SlabFwdArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  hipError_t e = allow_lds(k_slab_fwd<NT_SLAB, RS>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_slab_fwd<NT_SLAB, RS>), grid, dim3(NT_SLAB), lds, st, a);
  return hipGetLastError();
}
template hipError_t launch_slab_fwd<TB_RS>(const SlabFwdArgs& a, dim3 grid, size_t lds, hipStream_t st);
}  // namespace tb
