// Pass C: k_slab_inv -- per (bc, h) slab: inverse W, C2R along D, scale 1/N, zero D-padding,
// per-sample min/max epilogue.  Compiled once per radix set (-DTB_RS).  Body: pass_c_body.
#include "kernels.h"

namespace tb {
namespace {

template <int NT, int RS>
__global__ __launch_bounds__(NT) void k_slab_inv(SlabInvArgs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SlabInvArgs& a = kargs<SlabInvArgs>();
  DevCtx ctx{(int)threadIdx.x, NT};
  const int bc = a.bc0 + (int)blockIdx.y;
  float lo, hi;
  pass_c_body<DevCtx, RS>(ctx, reinterpret_cast<cf*>(smem), a.pl, a.S, a.y, a.sbc, a.sh, a.sw, a.ypad, bc,
                          (int)blockIdx.x, a.scale, &lo, &hi);
  if (a.mm) block_minmax_atomic<NT>(lo, hi, reinterpret_cast<float*>(smem), a.mm + 2 * (bc / a.C));
}
}  // namespace

template <int RS>
hipError_t launch_slab_inv(const SlabInvArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  hipError_t e = allow_lds(k_slab_inv<NT_SLAB, RS>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_slab_inv<NT_SLAB, RS>), grid, dim3(NT_SLAB), lds, st, a);
  return hipGetLastError();
}
template hipError_t launch_slab_inv<TB_RS>(const SlabInvArgs& a, dim3 grid, size_t lds, hipStream_t st);
}  // namespace tb
