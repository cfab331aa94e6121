// k_kspace_stats -- sum over the full spectrum of log(|k|+1e-10) after a sample's op program
// (KSpaceSpikeNoise default intensity, filters_and_operators.py:927-933).  Per radix set (-DTB_RS).
#include "kernels.h"

namespace tb {
namespace {
template <int NT, int RS>
__global__ __launch_bounds__(NT) void k_kspace_stats(StatsArgs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const StatsArgs& a = kargs<StatsArgs>();
  const tb_plan_dev& pl = a.pl;
  cf* lds = reinterpret_cast<cf*>(smem);
  DevCtx ctx{(int)threadIdx.x, NT};
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int T = a.T;
  const int H = pl.H, W = pl.W, D = pl.D, Dh = D / 2 + 1;
  const int ncols_all = W * Dh;
  const int j0 = (int)blockIdx.x * T;
  const int nc = (ncols_all - j0) < T ? (ncols_all - j0) : T;
  const TileGeo g = tile_geo(H, T);
  cf* tw = lds + g.off_tw;
  int* irev = reinterpret_cast<int*>(lds + g.off_irev);
  for (int i = threadIdx.x; i < H; i += NT) { tw[i] = pl.tw[0][i]; irev[i] = pl.irev_h[i]; }
  const cf* Sb = a.S + (int64_t)bc * H * ncols_all + j0;
  const int nl = H * nc;
  const FastDiv fnc = FastDiv::make(nc), fDh = FastDiv::make(Dh);
  for (int t = threadIdx.x; t < nl; t += NT) {
    const int hh = fnc.div(t), c = t - hh * nc;
    lds[hh * T + c] = Sb[(int64_t)hh * ncols_all + c];
  }
  __syncthreads();
  fft_dif<DevCtx, RS>(ctx, lds, tw, pl.ax[0], nc, TileAddr{T}, true);
  double acc = 0.0;
  const tb_sample_ops& so = a.ops.s[bcl / a.C];
  const int chan = bcl % a.C;
  const int Dtop = (D % 2 == 0) ? D / 2 : -1;
  for (int t = threadIdx.x; t < nl; t += NT) {
    const int hp = fnc.div(t), c = t - hp * nc;
    const int j = j0 + c;
    const int wp = fDh.div(j), kd = j - wp * Dh;
    const cf v = apply_ops(so, chan, lds[hp * T + c], freq_col(pl.irev_w[wp], kd, W, D), irev[hp], H);
    const float la = logf(f32_sqrt(v.x * v.x + v.y * v.y) + 1e-10f);
    acc += (kd == 0 || kd == Dtop) ? (double)la : 2.0 * (double)la;
  }
  // block reduce in double
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NT / 64; ++w) acc += red[w];
    atomicAdd(&a.out[bc], acc);
  }
}
}  // namespace

template <int RS>
hipError_t launch_kspace_stats(const StatsArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  hipError_t e = allow_lds(k_kspace_stats<NT_TILE, RS>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_kspace_stats<NT_TILE, RS>), grid, dim3(NT_TILE), lds, st, a);
  return hipGetLastError();
}
template hipError_t launch_kspace_stats<TB_RS>(const StatsArgs& a, dim3 grid, size_t lds, hipStream_t st);
}  // namespace tb
