// Pass B: k_kspace -- per (bc, tile of T spectrum columns): C2C along H (DIF), the sample's op
// program on every coefficient, inverse along H (DIT).  Compiled once per radix set (-DTB_RS).
#include "kernels.h"

namespace tb {
namespace {
template <int NT, int RS>
__global__ __launch_bounds__(NT) void k_kspace(KspaceArgs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const KspaceArgs& a = kargs<KspaceArgs>();
  DevCtx ctx{(int)threadIdx.x, NT};
  const int bcl = (int)blockIdx.y;
  pass_b_body<DevCtx, RS>(ctx, reinterpret_cast<cf*>(smem), a.pl, a.S, a.bc0 + bcl, (int)blockIdx.x, a.T,
                          a.ops.s[(a.cofs + bcl) / a.C], (a.cofs + bcl) % a.C);
}
}  // namespace

template <int RS>
hipError_t launch_kspace(const KspaceArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  hipError_t e = allow_lds(k_kspace<NT_TILE, RS>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_kspace<NT_TILE, RS>), grid, dim3(NT_TILE), lds, st, a);
  return hipGetLastError();
}
template hipError_t launch_kspace<TB_RS>(const KspaceArgs& a, dim3 grid, size_t lds, hipStream_t st);
}  // namespace tb
