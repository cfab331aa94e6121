// Pass B for the H extents with a compile-time plan (kspace_ct.h: H = 240, 128): per (bc, tile of
// 16 spectrum columns), one work item per thread per phase -- H stage 0 from HBM, the fused last
// DIF stage / op program / first DIT stage in registers, the inverse stage 0 back to HBM.
#include "kernels.h"
#include "kspace_ct.h"

namespace tb {

#ifdef TB_SLAB_PROF  // pass-B phase timestamps (as kern_slab_ct.hip)
__device__ unsigned long long g_kspace_prof[256][16][8];
#define TB_BSTAMP(U, I)                                                                        \
  do {                                                                                         \
    const int it_ = ((U) - (int)blockIdx.x) / (int)gridDim.x;                                  \
    if (threadIdx.x == 0 && blockIdx.x < 256 && it_ < 16)                                      \
      g_kspace_prof[blockIdx.x][it_][I] = __builtin_amdgcn_s_memtime();                        \
  } while (0)
#else
#define TB_BSTAMP(U, I) \
  do {                  \
  } while (0)
#endif

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

// Persistent paired variant: ncu x occupancy workgroups walk the (bc, tile) units u = blockIdx.x,
// + gridDim.x, ...; each unit's stage-0 inputs are loaded into registers while the previous unit
// runs its middle and inverse phases (one unit of HBM reads always in flight per workgroup, instead
// of every short-lived workgroup paying the HBM latency before any of its arithmetic starts).
template <int H, int T, int NT, int K>
__global__ __launch_bounds__(NT) void k_kspace_ct2p(KspaceArgs) {
  using P = ct::TilePlan<H, T>;
  static_assert(P::N0 / 2 <= NT && P::NM % NT == 0 && NT % T == 0, "paired items");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  const KspaceArgs& a = kargs<KspaceArgs>();
  const int tid = (int)threadIdx.x;
  const int ncols = a.pl.W * (a.pl.D / 2 + 1);
  const int ntile = ncols / T, units = ntile * a.nbc;
  const bool ld = tid < P::N0 / 2;
  for (int i = tid; i < H; i += NT) lds[P::OFF_TW + i] = ct::V(a.pl.tw[0][i].x, a.pl.tw[0][i].y);
  auto col0 = [&](int u, int& bcl) {
    bcl = u / ntile;
    return (u - bcl * ntile) * T;
  };
  ct::f4 r[P::Q0];
  int u = (int)blockIdx.x;
  if (u < units && ld) {
    int bcl;
    const int j0 = col0(u, bcl);
    ct::b_load_pair<P>(r, reinterpret_cast<const v2*>(a.S) + (int64_t)(a.bc0 + bcl) * H * ncols + j0, ncols, tid);
  }
  for (; u < units; u += (int)gridDim.x) {
    int bcl;
    const int j0 = col0(u, bcl);
    v2* Sc = reinterpret_cast<v2*>(a.S) + (int64_t)(a.bc0 + bcl) * H * ncols + j0;
    const FreqCol fc = ct::tile_col(a.pl, j0 + tid % T);
    TB_BSTAMP(u, 0);
    __syncthreads();  // the previous unit's inverse-stage reads of the tile are done (and the twiddles are in)
    TB_BSTAMP(u, 1);
    if (ld) ct::b_s0_pair_regs<P>(lds, r, tid);
    {  // the next unit's inputs, in flight during the middle and inverse phases (clamped on the last pass)
      const int un = u + (int)gridDim.x < units ? u + (int)gridDim.x : u;
      int bn;
      const int jn = col0(un, bn);
      if (ld) ct::b_load_pair<P>(r, reinterpret_cast<const v2*>(a.S) + (int64_t)(a.bc0 + bn) * H * ncols + jn, ncols, tid);
    }
    __syncthreads();
    TB_BSTAMP(u, 2);
    const int sl = a.cofs + bcl;
    if constexpr (K == ct::MASK_GENERIC) {
#pragma unroll 1
      for (int s = 0; s < P::NM / NT; ++s) ct::b_mid_lds<P>(lds, a.ops.s[sl / a.C], sl % a.C, fc, tid + s * NT);
    } else {
#pragma unroll 1
      for (int s = 0; s < P::NM / NT; ++s) ct::b_mid_mask<P, K>(lds, a.ops.s[sl / a.C], sl % a.C, fc, tid + s * NT);
    }
    __syncthreads();
    TB_BSTAMP(u, 3);
    if (ld) ct::b_s1_pair<P>(lds, Sc, ncols, tid);
    TB_BSTAMP(u, 4);
  }
}

// Persistent pass B over a split spectrum (kspace_ct.h b_mid_split): unit (bc, 16 first-half columns)
// with their 16 partner columns W/2 spectrum rows later, one 32-column tile; the next unit's loads are
// in flight during the middle and inverse phases (as k_kspace_ct2p).
template <int H, int W, int D, int NT, int K>
__global__ __launch_bounds__(NT) void k_kspace_half(KspaceArgs) {
  using HP = ct::HalfPlan<W, D>;
  using P = ct::TilePlan<H, 32>;
  constexpr int TH = 16;
  static_assert(P::N0 / 2 <= NT && (P::Q0 * TH) % NT == 0 && NT % TH == 0, "split tile items");
  static_assert((HP::W2 * HP::Dh) % TH == 0, "whole split tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  const KspaceArgs& a = kargs<KspaceArgs>();
  const int tid = (int)threadIdx.x;
  constexpr int ncols = W * HP::Dh, nh = HP::W2 * HP::Dh, ntile = nh / TH;
  const int units = ntile * a.nbc;
  const bool ld = tid < P::N0 / 2;
  for (int i = tid; i < H; i += NT) lds[P::OFF_TW + i] = ct::V(a.pl.tw[0][i].x, a.pl.tw[0][i].y);
  auto base = [&](int u, int& bcl) {
    bcl = u / ntile;
    return reinterpret_cast<v2*>(a.S) + (int64_t)(a.bc0 + bcl) * H * ncols + (u - bcl * ntile) * TH;
  };
  ct::f4 r[P::Q0];
  int u = (int)blockIdx.x;
  if (u < units && ld) {
    int bcl;
    ct::b_load_split<P>(r, base(u, bcl), ncols, nh, tid);
  }
  for (; u < units; u += (int)gridDim.x) {
    int bcl;
    v2* Sc = base(u, bcl);
    FreqCol f0, f1;
    ct::tile_col_half<HP>((u - bcl * ntile) * TH + tid % TH, f0, f1);
    __syncthreads();  // the previous unit's inverse-stage reads of the tile are done (and the twiddles are in)
    if (ld) ct::b_s0_pair_regs<P>(lds, r, tid);
    {
      const int un = u + (int)gridDim.x < units ? u + (int)gridDim.x : u;
      int bn;
      const v2* Sn = base(un, bn);
      if (ld) ct::b_load_split<P>(r, Sn, ncols, nh, tid);
    }
    __syncthreads();
    const int sl = a.cofs + bcl;
#pragma unroll 1
    for (int s = 0; s < P::Q0 * TH / NT; ++s)
      ct::b_mid_split<P, K>(lds, a.ops.s[sl / a.C], sl % a.C, f0, f1, tid + s * NT);
    __syncthreads();
    if (ld) ct::b_s1_split<P>(lds, Sc, ncols, nh, tid);
  }
}

}  // namespace

#ifdef TB_SLAB_PROF
extern "C" int tb_debug_kspace_prof(void* host, size_t bytes) {
  if (bytes > sizeof(g_kspace_prof)) bytes = sizeof(g_kspace_prof);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_kspace_prof), bytes, 0, hipMemcpyDeviceToHost);
}
#endif

bool kspace_ct_supported(int H) {
#define TB_X(h) if (H == h) return true;
  TB_CT_TILE_H(TB_X)
#undef TB_X
  return false;
}

// the paired kernel when every tile is full and rows stay 16-B aligned.  Tile width: 16 columns on
// 128-thread workgroups (4 per CU by LDS: 196 us per C3 launch; measured against 32 columns on 256
// threads, 2 per CU: 206 us, and 8 on 64 threads)
static bool use_pair(int ncols) {
  return ncols % ct::kCtTileT2 == 0;
}
static int pair_tile() {
  return 16;
}

int kspace_ct_tile(int ncols) { return use_pair(ncols) ? pair_tile() : ct::kCtTileT; }

// persistent pass B (measured against the one-tile-per-workgroup grid)
static bool use_persist() {
  return true;
}

template <class K>
static int kspace_occupancy(K kern, int nt, size_t lds) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(reinterpret_cast<const void*>(kern));
  if (it != cache.end()) return it->second;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, nt, lds) != hipSuccess || occ < 1) occ = 1;
  cache[reinterpret_cast<const void*>(kern)] = occ;
  return occ;
}

bool kspace_ct_persistent(int ncols) { return use_pair(ncols) && use_persist() && pair_tile() == 16; }

// the launch's programs all of one mask-op kind -> pass B's unrolled middle phase
// (else the generic one)
static int launch_mask_kind(const KspaceArgs& a) {
  if (a.nbc < 1) return ct::MASK_GENERIC;
  const int s0 = a.cofs / a.C, s1 = (a.cofs + a.nbc - 1) / a.C;
  return ct::mask_kind(a.ops.s + s0, s1 - s0 + 1);
}

hipError_t launch_kspace_ct(const KspaceArgs& a, dim3 grid, int ncu, hipStream_t st) {
  const bool pair = use_pair(a.pl.W * (a.pl.D / 2 + 1));
  if (pair && use_persist() && pair_tile() == 16) {
    const int mk = launch_mask_kind(a);
#define TB_X(h)                                                                           \
    if (a.pl.H == h) {                                                                    \
      constexpr size_t lds = ct::TilePlan<h, 16>::LDS_BYTES;                              \
      auto kern = mk == ct::MASK_GIBBS ? k_kspace_ct2p<h, 16, 128, ct::MASK_GIBBS>        \
                : mk == ct::MASK_LAYER ? k_kspace_ct2p<h, 16, 128, ct::MASK_LAYER>        \
                : mk == ct::MASK_DISK  ? k_kspace_ct2p<h, 16, 128, ct::MASK_DISK>         \
                                       : k_kspace_ct2p<h, 16, 128, ct::MASK_GENERIC>;     \
      hipError_t e = allow_lds(kern, lds);                                                \
      if (e != hipSuccess) return e;                                                      \
      const int units = (int)(grid.x * grid.y);                                           \
      int g = ncu * kspace_occupancy(kern, 128, lds);                                     \
      g = g < units ? g : units;                                                          \
      hipLaunchKernelGGL(kern, dim3(g), dim3(128), lds, st, a);                           \
      return hipGetLastError();                                                           \
    }
    TB_CT_TILE_H(TB_X)
#undef TB_X
  }
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

bool kspace_half_supported(int H, int W, int D) {
  if (H != 240) return false;
#define TB_X(w, d) if (W == w && D == d) return true;
  TB_CT_HALF_SHAPES(TB_X)
#undef TB_X
  return false;
}

hipError_t launch_kspace_half(const KspaceArgs& a, int ncu, hipStream_t st) {
  const int mk = launch_mask_kind(a);
#define TB_X(w, d)                                                                                   \
  if (a.pl.H == 240 && a.pl.W == w && a.pl.D == d) {                                                 \
    constexpr size_t lds = ct::TilePlan<240, 32>::LDS_BYTES;                                         \
    auto kern = mk == ct::MASK_GIBBS ? k_kspace_half<240, w, d, 256, ct::MASK_GIBBS>                 \
              : mk == ct::MASK_LAYER ? k_kspace_half<240, w, d, 256, ct::MASK_LAYER>                 \
              : mk == ct::MASK_DISK  ? k_kspace_half<240, w, d, 256, ct::MASK_DISK>                  \
                                     : k_kspace_half<240, w, d, 256, ct::MASK_GENERIC>;              \
    hipError_t e = allow_lds(kern, lds);                                                             \
    if (e != hipSuccess) return e;                                                                   \
    const int units = (w / 2) * (d / 2 + 1) / 16 * a.nbc;                                           \
    int g = ncu * kspace_occupancy(kern, 256, lds);                                                  \
    g = g < units ? g : units;                                                                       \
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), lds, st, a);                                        \
    return hipGetLastError();                                                                        \
  }
  TB_CT_HALF_SHAPES(TB_X)
#undef TB_X
  return hipErrorInvalidValue;
}

}  // namespace tb
