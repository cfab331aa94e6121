// Pass B for the H extents with a compile-time plan (kspace_ct.h: H = 240, 128): per (bc, tile of
// 16 spectrum columns), one work item per thread per phase -- H stage 0 from HBM, the fused last
// DIF stage / op program / first DIT stage in registers, the inverse stage 0 back to HBM.
#include "kernels.h"
#include "kspace_ct.h"

namespace tb {
namespace {
using ct::v2;

template <int H, int T, int NT>
__global__ __launch_bounds__(NT) void k_kspace_ct(KspaceArgs) {
  using P = ct::TilePlan<H, T>;
  static_assert(P::N0 <= NT && P::NM <= NT, "one item per thread per phase");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  const KspaceArgs& a = kargs<KspaceArgs>();
  const int tid = (int)threadIdx.x;
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int ncols = a.pl.W * (a.pl.D / 2 + 1);
  const int j0 = (int)blockIdx.x * T;
  const int nc = (ncols - j0) < T ? (ncols - j0) : T;
  v2* Sc = reinterpret_cast<v2*>(a.S) + (int64_t)bc * H * ncols + j0;
  const bool act = tid < P::N0 && (tid % T) < nc;
  v2 r[P::Q0];
#pragma unroll
  for (int q = 0; q < P::Q0; ++q) r[q] = ct::V(0.f, 0.f);
  if (act) ct::b_load<P>(r, Sc, ncols, tid);
  for (int i = tid; i < H; i += NT) lds[P::OFF_TW + i] = ct::V(a.pl.tw[0][i].x, a.pl.tw[0][i].y);
  __syncthreads();
  if (tid < P::N0) ct::b_s0<P>(lds, r, tid);
  __syncthreads();
  if (tid < P::NM) {
    const int c = tid % T;
    const FreqCol fc = ct::tile_col(a.pl, j0 + (c < nc ? c : 0));
    ct::b_mid<P>(lds, a.ops.s[(a.cofs + bcl) / a.C], (a.cofs + bcl) % a.C, fc, tid);
  }
  __syncthreads();
  if (act) ct::b_s1<P>(lds, Sc, ncols, tid);
}

// Paired variant (ncols even, ncols % T == 0): stage-0 items cover two adjacent columns, so the
// HBM loads / stores are 16 B per lane; the middle phase runs NM / NT items per thread.
template <int H, int T, int NT>
__global__ __launch_bounds__(NT) void k_kspace_ct2(KspaceArgs) {
  using P = ct::TilePlan<H, T>;
  static_assert(P::N0 / 2 <= NT && P::NM % NT == 0, "paired items: one per thread per stage-0 phase");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  const KspaceArgs& a = kargs<KspaceArgs>();
  const int tid = (int)threadIdx.x;
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int ncols = a.pl.W * (a.pl.D / 2 + 1);
  const int j0 = (int)blockIdx.x * T;
  v2* Sc = reinterpret_cast<v2*>(a.S) + (int64_t)bc * H * ncols + j0;
  // the middle phase's column geometry (its w' -> kw table read is a dependent global load):
  // formed before the stage-0 loads so its latency hides under theirs; NT % T == 0, so every
  // middle item of this thread has tile column tid % T
  static_assert(NT % T == 0, "one tile column per thread in the middle phase");
  const FreqCol fc = ct::tile_col(a.pl, j0 + tid % T);
  for (int i = tid; i < H; i += NT) lds[P::OFF_TW + i] = ct::V(a.pl.tw[0][i].x, a.pl.tw[0][i].y);
  __syncthreads();
  if (tid < P::N0 / 2) ct::b_s0_pair<P>(lds, Sc, ncols, tid);
  __syncthreads();
  const int sl = a.cofs + bcl;
#pragma unroll
  for (int s = 0; s < P::NM / NT; ++s) ct::b_mid<P>(lds, a.ops.s[sl / a.C], sl % a.C, fc, tid + s * NT);
  __syncthreads();
  if (tid < P::N0 / 2) ct::b_s1_pair<P>(lds, Sc, ncols, tid);
}

}  // namespace

bool kspace_ct_supported(int H) {
#define TB_X(h) if (H == h) return true;
  TB_CT_TILE_H(TB_X)
#undef TB_X
  return false;
}

// the paired kernel when every tile is full and rows stay 16-B aligned.  Tile width (TEXBIAS_KSPACE_T2):
// 16 columns on 128-thread workgroups by default (4 per CU by LDS: 196 us per C3 launch), 32 on
// 256 threads (2 per CU: 206 us), or 8 on 64 threads
static bool use_pair(int ncols) {
  static const bool on = [] {
    const char* e = std::getenv("TEXBIAS_KSPACE_PAIR");
    return !(e && std::atoi(e) == 0);
  }();
  return on && ncols % ct::kCtTileT2 == 0;
}
static int pair_tile() {
  static const int t = [] {
    const char* e = std::getenv("TEXBIAS_KSPACE_T2");
    const int v = e ? std::atoi(e) : 16;
    return (v == 8 || v == 32) ? v : 16;
  }();
  return t;
}

int kspace_ct_tile(int ncols) { return use_pair(ncols) ? pair_tile() : ct::kCtTileT; }

hipError_t launch_kspace_ct(const KspaceArgs& a, dim3 grid, hipStream_t st) {
  const bool pair = use_pair(a.pl.W * (a.pl.D / 2 + 1));
#define TB_X(h)                                                                         \
  if (a.pl.H == h && pair && pair_tile() == 8) {                                        \
    constexpr size_t lds = ct::TilePlan<h, 8>::LDS_BYTES;                               \
    hipError_t e = allow_lds(k_kspace_ct2<h, 8, 64>, lds);                              \
    if (e != hipSuccess) return e;                                                      \
    hipLaunchKernelGGL((k_kspace_ct2<h, 8, 64>), grid, dim3(64), lds, st, a);           \
    return hipGetLastError();                                                           \
  }                                                                                     \
  if (a.pl.H == h && pair && pair_tile() == 16) {                                       \
    constexpr size_t lds = ct::TilePlan<h, 16>::LDS_BYTES;                              \
    hipError_t e = allow_lds(k_kspace_ct2<h, 16, 128>, lds);                            \
    if (e != hipSuccess) return e;                                                      \
    hipLaunchKernelGGL((k_kspace_ct2<h, 16, 128>), grid, dim3(128), lds, st, a);        \
    return hipGetLastError();                                                           \
  }                                                                                     \
  if (a.pl.H == h && pair) {                                                            \
    constexpr size_t lds = ct::TilePlan<h, ct::kCtTileT2>::LDS_BYTES;                   \
    hipError_t e = allow_lds(k_kspace_ct2<h, ct::kCtTileT2, NT_TILE>, lds);             \
    if (e != hipSuccess) return e;                                                      \
    hipLaunchKernelGGL((k_kspace_ct2<h, ct::kCtTileT2, NT_TILE>), grid, dim3(NT_TILE), lds, st, a); \
    return hipGetLastError();                                                           \
  }                                                                                     \
  if (a.pl.H == h) {                                                                    \
    constexpr size_t lds = ct::TilePlan<h, ct::kCtTileT>::LDS_BYTES;                    \
    hipError_t e = allow_lds(k_kspace_ct<h, ct::kCtTileT, NT_TILE>, lds);               \
    if (e != hipSuccess) return e;                                                      \
    hipLaunchKernelGGL((k_kspace_ct<h, ct::kCtTileT, NT_TILE>), grid, dim3(NT_TILE), lds, st, a); \
    return hipGetLastError();                                                           \
  }
  TB_CT_TILE_H(TB_X)
#undef TB_X
  return hipErrorInvalidValue;
}

}  // namespace tb
