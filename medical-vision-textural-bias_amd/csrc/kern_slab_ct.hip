// Passes A / C for the slab shapes with a compile-time plan (slab_ct.h: W x D = 240 x 155, 128 x 128).
//
// One 150 KB slab fills a CU's LDS, so a workgroup cannot overlap its HBM traffic with another
// workgroup's FFT work on the same CU.  These kernels are therefore persistent (one workgroup per
// CU walks the (bc, h) units u = blockIdx.x, +gridDim.x, ...) and software-pipelined: the
// first-stage inputs of unit u + gridDim.x (pass A: 2*R0 floats per item, pass C: Q1 complex per
// item) are loaded into registers during the last phases of unit u (after the register-heavy
// prime-radix and unpack phases, so they do not raise the peak register count), and the last stage
// of each unit writes HBM straight from registers.  Phases inside a unit are barrier-separated (slab_ct.h lists them).
#include "kernels.h"
#include "slab_ct.h"

namespace tb {

// Phase timestamps (measurement builds only: -DTB_SLAB_PROF, scripts/build_variant.sh): thread 0 of
// workgroups < 256 stamps the shader clock after each barrier of its first 16 units.
#ifdef TB_SLAB_PROF
__device__ unsigned long long g_slab_prof[2][256][16][12];
#define TB_STAMP(K, U, I)                                                                      \
  do {                                                                                         \
    const int it_ = ((U) - (int)blockIdx.x) / (int)gridDim.x;                                  \
    if (threadIdx.x == 0 && blockIdx.x < 256 && it_ < 16)                                      \
      g_slab_prof[K][blockIdx.x][it_][I] = __builtin_amdgcn_s_memtime();                       \
  } while (0)
#else
#define TB_STAMP(K, U, I) \
  do {                    \
  } while (0)
#endif

namespace {
using ct::v2;

template <int W, int D, int NT, bool FUSE>
__global__ __launch_bounds__(NT) void k_slab_fwd_ct(SlabFwdArgs) {
  using P = ct::SlabPlan<W, D>;
  constexpr int SF = ct::Slots<P::N_F0, NT>::value;
  constexpr int SU = ct::Slots<P::N_U, NT>::value;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  const SlabFwdArgs& a = kargs<SlabFwdArgs>();
  const int tid = (int)threadIdx.x;
  const int H = a.pl.H, units = H * a.nbc;
  DevCtx ctx{tid, NT};
  ct::load_tw<P>(ctx, lds, a.pl);
  v2 rf[SF][P::R0];
  int u = (int)blockIdx.x;
  if (u < units) {
    const int bcl = u / H, h = u - bcl * H;
    const float* xb = a.x + (int64_t)(a.bc0 + bcl) * a.sbc + (int64_t)h * a.sh;
#pragma unroll
    for (int s = 0; s < SF; ++s)
      if (tid + s * NT < P::N_F0) ct::a_load<P>(rf[s], xb, a.sw, tid + s * NT);
  }
  for (; u < units; u += (int)gridDim.x) {
    __syncthreads();  // the previous unit's W1 reads are done (and the twiddles are visible)
#pragma unroll
    for (int s = 0; s < SF; ++s)
      if (tid + s * NT < P::N_F0) ct::a_f0<P>(lds, rf[s], tid + s * NT);
    __syncthreads();
    if constexpr (FUSE && P::FUSED_DU) {  // D stage 1 + unpack in one phase (slab_ct.h a_du_*)
      constexpr int SD = ct::Slots<P::N_DU, NT>::value;
      v2 rd[SD][2 * P::R1];
#pragma unroll
      for (int s = 0; s < SD; ++s)
        if (tid + s * NT < P::N_DU) ct::a_du_load<P>(lds, rd[s], tid + s * NT);
      __syncthreads();
#pragma unroll
      for (int s = 0; s < SD; ++s)
        if (tid + s * NT < P::N_DU) ct::a_du_compute<P>(lds, rd[s], tid + s * NT);
    } else {
      _Pragma("unroll 1") for (int it = tid; it < P::N_D1; it += NT) ct::a_d1<P>(lds, it);
      __syncthreads();
      v2 ru[SU][2];
#pragma unroll
      for (int s = 0; s < SU; ++s)
        if (tid + s * NT < P::N_U) ct::a_u_read<P>(lds, ru[s], tid + s * NT);
      __syncthreads();
#pragma unroll
      for (int s = 0; s < SU; ++s)
        if (tid + s * NT < P::N_U) ct::a_u_write<P>(lds, ru[s], tid + s * NT);
    }
    const int un = u + (int)gridDim.x;
    {  // next unit's first-stage inputs, in flight during W0 / W1 below (unconditional -- a clamped
       // unit on the last pass -- so the consumed registers are dead, not carried by a phi)
      const int uc = un < units ? un : u;
      const int bcl = uc / H, h = uc - bcl * H;
      const float* xb = a.x + (int64_t)(a.bc0 + bcl) * a.sbc + (int64_t)h * a.sh;
#pragma unroll
      for (int s = 0; s < SF; ++s)
        if (tid + s * NT < P::N_F0) ct::a_load<P>(rf[s], xb, a.sw, tid + s * NT);
    }
    __syncthreads();
    _Pragma("unroll 1") for (int it = tid; it < P::N_W0; it += NT) ct::a_w0<P>(lds, it);
    __syncthreads();
    const int bcl = u / H, h = u - bcl * H;
    v2* Sb = reinterpret_cast<v2*>(a.S) + ((int64_t)(a.bc0 + bcl) * H + h) * (int64_t)(W * P::Dh);
    _Pragma("unroll 1") for (int it = tid; it < P::N_W1; it += NT) ct::a_w1<P>(lds, Sb, it);
  }
}

// Pass A with 16-B loads (contiguous slabs: sw == D, 16-B aligned): the next unit's whole raw
// slab is prefetched as float4 lanes during W0 / W1 (instead of 4-B lanes in F0 item order, which
// cost ~110 of the ~280 us per C3 launch), written to LDS at the start of the unit (raw rows 2p,
// 2p+1 are the bytes of pair row p of Z), then F0 reads its inputs from there.
template <int W, int D, int NT, bool EARLY>
__global__ __launch_bounds__(NT) void k_slab_fwd_ct16(SlabFwdArgs) {
  using P = ct::SlabPlan<W, D>;
  static_assert((W * D) % 4 == 0, "whole float4 slabs");
  constexpr int NV = W * D / 4;
  constexpr int SV = ct::Slots<NV, NT>::value;
  constexpr int SF = ct::Slots<P::N_F0, NT>::value;
  constexpr int SU = ct::Slots<P::N_U, NT>::value;
  typedef float f4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  const SlabFwdArgs& a = kargs<SlabFwdArgs>();
  const int tid = (int)threadIdx.x;
  const int H = a.pl.H, units = H * a.nbc;
  DevCtx ctx{tid, NT};
  ct::load_tw<P>(ctx, lds, a.pl);
  f4 rv[SV];
  int u = (int)blockIdx.x;
  if (u < units) {
    const int bcl = u / H, h = u - bcl * H;
    const f4* xb = reinterpret_cast<const f4*>(a.x + (int64_t)(a.bc0 + bcl) * a.sbc + (int64_t)h * a.sh);
#pragma unroll
    for (int s = 0; s < SV; ++s)
      if (tid + s * NT < NV) rv[s] = ld_stream<TB_NT_LOADS>(xb + tid + s * NT);
  }
  for (; u < units; u += (int)gridDim.x) {
    TB_STAMP(0, u, 0);
    __syncthreads();  // the previous unit's W1 reads are done (and the twiddles are visible)
    TB_STAMP(0, u, 1);
    {
      f4* raw4 = reinterpret_cast<f4*>(smem);
#pragma unroll
      for (int s = 0; s < SV; ++s)
        if (tid + s * NT < NV) raw4[tid + s * NT] = rv[s];
    }
    __syncthreads();
    TB_STAMP(0, u, 2);
    v2 rf[SF][P::R0];
#pragma unroll
    for (int s = 0; s < SF; ++s)
      if (tid + s * NT < P::N_F0) ct::a_load_raw<P>(reinterpret_cast<const float*>(smem), rf[s], tid + s * NT);
    __syncthreads();  // every raw read is done before Z (the same bytes) is written
    TB_STAMP(0, u, 3);
#pragma unroll
    for (int s = 0; s < SF; ++s)
      if (tid + s * NT < P::N_F0) ct::a_f0<P>(lds, rf[s], tid + s * NT);
    // next unit's raw slab (clamped on the last pass, as in k_slab_fwd_ct): EARLY issues it here,
    // in flight during D1 / U / W0 / W1, else after U (in flight during W0 / W1 only)
    // (issuing these loads spread over F0 / D1 / U / W0 instead measured no faster: the F0 phase
    // shrank by what the later phases grew, and the kernel spilled)
    auto prefetch = [&]() {
      const int un = u + (int)gridDim.x;
      const int uc = un < units ? un : u;
      const int bcl = uc / H, h = uc - bcl * H;
      const f4* xb = reinterpret_cast<const f4*>(a.x + (int64_t)(a.bc0 + bcl) * a.sbc + (int64_t)h * a.sh);
#pragma unroll
      for (int s = 0; s < SV; ++s)
        if (tid + s * NT < NV) rv[s] = ld_stream<TB_NT_LOADS>(xb + tid + s * NT);
    };
    if constexpr (EARLY) prefetch();
    __syncthreads();
    TB_STAMP(0, u, 4);
    _Pragma("unroll 1") for (int it = tid; it < P::N_D1; it += NT) ct::a_d1<P>(lds, it);
    __syncthreads();
    TB_STAMP(0, u, 5);
    {
      v2 ru[SU][2];
#pragma unroll
      for (int s = 0; s < SU; ++s)
        if (tid + s * NT < P::N_U) ct::a_u_read<P>(lds, ru[s], tid + s * NT);
      __syncthreads();
      TB_STAMP(0, u, 6);
#pragma unroll
      for (int s = 0; s < SU; ++s)
        if (tid + s * NT < P::N_U) ct::a_u_write<P>(lds, ru[s], tid + s * NT);
    }
    if constexpr (!EARLY) prefetch();
    __syncthreads();
    TB_STAMP(0, u, 7);
    _Pragma("unroll 1") for (int it = tid; it < P::N_W0; it += NT) ct::a_w0<P>(lds, it);
    __syncthreads();
    TB_STAMP(0, u, 8);
    const int bcl = u / H, h = u - bcl * H;
    v2* Sb = reinterpret_cast<v2*>(a.S) + ((int64_t)(a.bc0 + bcl) * H + h) * (int64_t)(W * P::Dh);
    // (W1 in place in LDS + one contiguous 16-B sweep of the slab's spectrum, every line written
    // whole, measured 13 us slower per C3 launch than these strided 8-B stores)
    _Pragma("unroll 1") for (int it = tid; it < P::N_W1; it += NT) ct::a_w1<P>(lds, Sb, it);
    TB_STAMP(0, u, 9);
  }
}

template <int W, int D, int NT, bool FUSE>
__global__ __launch_bounds__(NT) void k_slab_inv_ct(SlabInvArgs) {
  using P = ct::SlabPlan<W, D>;
  constexpr int SG = ct::Slots<P::N_W1, NT>::value;
  constexpr int SU = ct::Slots<P::N_U, NT>::value;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[2 * NT / 64];
  v2* lds = reinterpret_cast<v2*>(smem);
  const SlabInvArgs& a = kargs<SlabInvArgs>();
  const int tid = (int)threadIdx.x;
  const int H = a.pl.H, units = H * a.nbc;
  const int64_t sstride = (int64_t)W * P::Dh;
  DevCtx ctx{tid, NT};
  ct::load_tw<P>(ctx, lds, a.pl);
  v2 rg[SG][P::Q1];
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  int u = (int)blockIdx.x;
  if (u < units) {
    const v2* Sb = reinterpret_cast<const v2*>(a.S) + ((int64_t)a.bc0 * H + u) * sstride;
#pragma unroll
    for (int s = 0; s < SG; ++s)
      if (tid + s * NT < P::N_W1) ct::c_load<P>(rg[s], Sb, tid + s * NT);
  }
  for (; u < units; u += (int)gridDim.x) {
    TB_STAMP(1, u, 0);
    __syncthreads();  // the previous unit's E0 reads are done
    TB_STAMP(1, u, 1);
#pragma unroll
    for (int s = 0; s < SG; ++s)
      if (tid + s * NT < P::N_W1) ct::c_g0<P>(lds, rg[s], tid + s * NT);
    __syncthreads();
    TB_STAMP(1, u, 2);
    _Pragma("unroll 1") for (int it = tid; it < P::N_W0; it += NT) ct::c_g1<P>(lds, it);
    __syncthreads();
    TB_STAMP(1, u, 3);
    if constexpr (FUSE && P::FUSED_DU) {  // repack + inverse D stage 1 in one phase (slab_ct.h c_re_*)
      constexpr int SD = ct::Slots<P::N_DU, NT>::value;
      v2 rd[SD][2 * P::R1];
#pragma unroll
      for (int s = 0; s < SD; ++s)
        if (tid + s * NT < P::N_DU) ct::c_re_load<P>(lds, rd[s], tid + s * NT);
      __syncthreads();
      TB_STAMP(1, u, 4);
#pragma unroll
      for (int s = 0; s < SD; ++s)
        if (tid + s * NT < P::N_DU) ct::c_re_compute<P>(lds, rd[s], tid + s * NT);
    } else {
      v2 ru[SU][2];
#pragma unroll
      for (int s = 0; s < SU; ++s)
        if (tid + s * NT < P::N_U) ct::c_r_read<P>(lds, ru[s], tid + s * NT);
      __syncthreads();
#pragma unroll
      for (int s = 0; s < SU; ++s)
        if (tid + s * NT < P::N_U) ct::c_r_write<P>(lds, ru[s], tid + s * NT);
      __syncthreads();
      _Pragma("unroll 1") for (int it = tid; it < P::N_D1; it += NT) ct::c_e1<P>(lds, it);
    }
    const int un = u + (int)gridDim.x;
    {  // next unit's first-stage inputs, in flight during E0 below (unconditional, as in pass A)
      const v2* Sb = reinterpret_cast<const v2*>(a.S) + ((int64_t)a.bc0 * H + (un < units ? un : u)) * sstride;
#pragma unroll
      for (int s = 0; s < SG; ++s)
        if (tid + s * NT < P::N_W1) ct::c_load<P>(rg[s], Sb, tid + s * NT);
    }
    __syncthreads();
    TB_STAMP(1, u, 5);
    const int bcl = u / H, h = u - bcl * H, bc = a.bc0 + bcl;
    float* yb = a.y + (int64_t)bc * a.sbc + (int64_t)h * a.sh;
    _Pragma("unroll 1") for (int it = tid; it < P::N_F0; it += NT) ct::c_e0<P>(lds, yb, a.sw, a.scale, it, lo, hi);
    TB_STAMP(1, u, 6);
    if (a.ypad > 0) {
      const FastDiv fp = FastDiv::make(a.ypad);
      for (int t = tid; t < W * a.ypad; t += NT) {
        const int w = fp.div(t);
        yb[(int64_t)w * a.sw + D + (t - w * a.ypad)] = 0.f;
      }
    }
    // flush the running min/max when the next unit belongs to another sample (or there is none)
    const int b = bc / a.C;
    if (a.mm && (un >= units || (a.bc0 + un / H) / a.C != b)) {
      block_minmax_atomic<NT>(lo, hi, red, a.mm + 2 * b);
      lo = 3.402823466e38f;
      hi = -3.402823466e38f;
    }
    TB_STAMP(1, u, 7);
  }
}

// ---------------------------------------------------------------- half units (slab_ct.h HalfPlan)
typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// block -> (slab, parity): blocks b and b + 8 hold the two halves of one slab -- the same XCD (blocks
// go to the XCDs round robin) at nearly the same time, so the 128-B lines their row ends share are
// fetched (pass A) or merged (pass C) once in that XCD's L2
__device__ __forceinline__ void half_unit(int b, int& slab, int& e) {
  slab = (b >> 4) * 8 + (b & 7);
  e = (b >> 3) & 1;
}
static int half_grid(int units) { return 16 * ((units + 7) / 8); }

// Pass A of one half unit: rows 2 w'' + e staged raw[w''][d] by 4-B global->LDS DMA (no registers:
// the other workgroup on the CU computes while these land), then F0 / D1+U (or fused DU) / W0 / W1
// with the SlabPlan<W/2, D> items, W1 storing the unit's split rows (e = 1 scaled by w^k'').
template <int W, int D, int NT, bool FUSE>
__global__ __launch_bounds__(NT) void k_slab_fwd_half(SlabFwdArgs) {
  using HP = ct::HalfPlan<W, D>;
  using P = typename HP::P;
  constexpr int SF = ct::Slots<P::N_F0, NT>::value;
  constexpr int SU = ct::Slots<P::N_U, NT>::value;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  v2* lds = reinterpret_cast<v2*>(smem);
  float* raw = reinterpret_cast<float*>(smem);
  const SlabFwdArgs& a = kargs<SlabFwdArgs>();
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.pl.H, units = H * a.nbc;
  int slab, e;
  half_unit((int)blockIdx.x, slab, e);
  if (slab >= units) return;
  const int bcl = slab / H, h = slab - bcl * H;
  const float* xb = a.x + (int64_t)(a.bc0 + bcl) * a.sbc + (int64_t)h * a.sh + (int64_t)e * a.sw;
  const int64_t sw2 = 2 * a.sw;
  {
    constexpr int NCH = (HP::NRAW + 63) / 64;
    for (int c = wave; c < NCH; c += NT / 64) {
      const int L = c * 64 + lane;
      if (L < HP::NRAW) {
        const int w2 = L / D, d = L - w2 * D;
        __builtin_amdgcn_global_load_lds((gptr_t)(xb + w2 * sw2 + d), (lptr_t)(raw + c * 64), 4, 0, 0);
      }
    }
  }
  DevCtx ctx{tid, NT};
  ct::load_tw_half<HP>(ctx, lds, a.pl);
  __syncthreads();  // vmcnt(0): the staged rows have landed
  {
    v2 rf[SF][P::R0];
#pragma unroll
    for (int s = 0; s < SF; ++s)
      if (tid + s * NT < P::N_F0) ct::a_load_raw<P>(raw, rf[s], tid + s * NT);
    __syncthreads();  // raw is the bytes of Z
#pragma unroll
    for (int s = 0; s < SF; ++s)
      if (tid + s * NT < P::N_F0) ct::a_f0<P>(lds, rf[s], tid + s * NT);
  }
  __syncthreads();
  if constexpr (FUSE && P::FUSED_DU) {
    constexpr int SD = ct::Slots<P::N_DU, NT>::value;
    v2 rd[SD][2 * P::R1];
#pragma unroll
    for (int s = 0; s < SD; ++s)
      if (tid + s * NT < P::N_DU) ct::a_du_load<P>(lds, rd[s], tid + s * NT);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SD; ++s)
      if (tid + s * NT < P::N_DU) ct::a_du_compute<P>(lds, rd[s], tid + s * NT);
  } else {
    _Pragma("unroll 1") for (int it = tid; it < P::N_D1; it += NT) ct::a_d1<P>(lds, it);
    __syncthreads();
    v2 ru[SU][2];
#pragma unroll
    for (int s = 0; s < SU; ++s)
      if (tid + s * NT < P::N_U) ct::a_u_read<P>(lds, ru[s], tid + s * NT);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SU; ++s)
      if (tid + s * NT < P::N_U) ct::a_u_write<P>(lds, ru[s], tid + s * NT);
  }
  __syncthreads();
  _Pragma("unroll 1") for (int it = tid; it < P::N_W0; it += NT) ct::a_w0<P>(lds, it);
  __syncthreads();
  v2* Sb = reinterpret_cast<v2*>(a.S) + ((int64_t)(a.bc0 + bcl) * H + h) * (int64_t)(W * P::Dh) +
           (int64_t)e * HP::W2 * P::Dh;
  _Pragma("unroll 1") for (int it = tid; it < P::N_W1; it += NT) ct::a_w1_half<HP>(lds, Sb, e, it);
}

// Pass C of one half unit: the unit's split rows (e = 1 scaled by w^-k'') -> inverse W/2-point DFT ->
// C2R along D -> rows 2 w'' + e of the image, zero padding, min/max
template <int W, int D, int NT, bool FUSE>
__global__ __launch_bounds__(NT) void k_slab_inv_half(SlabInvArgs) {
  using HP = ct::HalfPlan<W, D>;
  using P = typename HP::P;
  constexpr int SG = ct::Slots<P::N_W1, NT>::value;
  constexpr int SU = ct::Slots<P::N_U, NT>::value;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[2 * NT / 64];
  v2* lds = reinterpret_cast<v2*>(smem);
  const SlabInvArgs& a = kargs<SlabInvArgs>();
  const int tid = (int)threadIdx.x;
  const int H = a.pl.H, units = H * a.nbc;
  int slab, e;
  half_unit((int)blockIdx.x, slab, e);
  if (slab >= units) return;
  const int bcl = slab / H, h = slab - bcl * H, bc = a.bc0 + bcl;
  const v2* Sb = reinterpret_cast<const v2*>(a.S) + ((int64_t)bc * H + h) * (int64_t)(W * P::Dh) +
                 (int64_t)e * HP::W2 * P::Dh;
  {
    v2 rg[SG][P::Q1];
#pragma unroll
    for (int s = 0; s < SG; ++s)
      if (tid + s * NT < P::N_W1) ct::c_load_half<HP>(rg[s], Sb, tid + s * NT);
    DevCtx ctx{tid, NT};
    ct::load_tw_half<HP>(ctx, lds, a.pl);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SG; ++s)
      if (tid + s * NT < P::N_W1) {
        ct::c_twiddle_half<HP>(lds, rg[s], e, tid + s * NT);
        ct::c_g0<P>(lds, rg[s], tid + s * NT);
      }
  }
  __syncthreads();
  _Pragma("unroll 1") for (int it = tid; it < P::N_W0; it += NT) ct::c_g1<P>(lds, it);
  __syncthreads();
  if constexpr (FUSE && P::FUSED_DU) {
    constexpr int SD = ct::Slots<P::N_DU, NT>::value;
    v2 rd[SD][2 * P::R1];
#pragma unroll
    for (int s = 0; s < SD; ++s)
      if (tid + s * NT < P::N_DU) ct::c_re_load<P>(lds, rd[s], tid + s * NT);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SD; ++s)
      if (tid + s * NT < P::N_DU) ct::c_re_compute<P>(lds, rd[s], tid + s * NT);
  } else {
    v2 ru[SU][2];
#pragma unroll
    for (int s = 0; s < SU; ++s)
      if (tid + s * NT < P::N_U) ct::c_r_read<P>(lds, ru[s], tid + s * NT);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SU; ++s)
      if (tid + s * NT < P::N_U) ct::c_r_write<P>(lds, ru[s], tid + s * NT);
    __syncthreads();
    _Pragma("unroll 1") for (int it = tid; it < P::N_D1; it += NT) ct::c_e1<P>(lds, it);
  }
  __syncthreads();
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  float* yb = a.y + (int64_t)bc * a.sbc + (int64_t)h * a.sh + (int64_t)e * a.sw;
  const int64_t sw2 = 2 * a.sw;
  _Pragma("unroll 1") for (int it = tid; it < P::N_F0; it += NT) ct::c_e0<P>(lds, yb, sw2, a.scale, it, lo, hi);
  if (a.ypad > 0) {
    const FastDiv fp = FastDiv::make(a.ypad);
    for (int t = tid; t < HP::W2 * a.ypad; t += NT) {
      const int w = fp.div(t);
      yb[(int64_t)w * sw2 + D + (t - w * a.ypad)] = 0.f;
    }
  }
  if (a.mm) block_minmax_atomic<NT>(lo, hi, red, a.mm + 2 * (bc / a.C));
}

int slab_grid(int units, size_t lds, int ncu) {
  int per_cu = (int)(163840 / (lds ? lds : 1));
  per_cu = per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu);
  const int g = ncu * per_cu;
  return units < g ? units : g;
}

template <class K, class A>
hipError_t launch_ct(K kern, int nt, size_t lds, int units, int ncu, const A& a, hipStream_t st) {
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(slab_grid(units, lds, ncu)), dim3(nt), lds, st, a);
  return hipGetLastError();
}

}  // namespace

#ifdef TB_SLAB_PROF
extern "C" int tb_debug_slab_prof(void* host, size_t bytes) {
  if (bytes > sizeof(g_slab_prof)) bytes = sizeof(g_slab_prof);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_slab_prof), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int tb_debug_slab_prof_clear() {
  static unsigned long long z[2][256][16][12];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_slab_prof), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#endif

// threads per workgroup: 768 (3 waves per SIMD; measured against 512).  The fused DU / RE phase variant
// (slab_ct.h) is used for the inverse pass only (bit 2): it holds two butterflies' inputs across a
// barrier, which fits the register file only at 2 waves per SIMD.
static int ct_nt() {
  return 768;
}
static int ct_fuse() {
  return 2;
}

bool slab_ct_supported(int W, int D) {
#define TB_X(w, d) if (W == w && D == d) return true;
  TB_CT_SLAB_SHAPES(TB_X)
#undef TB_X
  return false;
}

// 16-B staged loads when the slabs are contiguous and 16-B aligned
static bool raw16_ok(const SlabFwdArgs& a) {
  return a.sw == a.pl.D && a.sh % 4 == 0 && a.sbc % 4 == 0 && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0 &&
         (a.pl.W * a.pl.D) % 4 == 0 && (reinterpret_cast<uintptr_t>(a.S) & 15) == 0;
}

static bool raw16_early() {
  return true;
}

hipError_t launch_slab_fwd_ct(const SlabFwdArgs& a, int ncu, hipStream_t st) {
  const int units = a.pl.H * a.nbc;
  const bool r16 = raw16_ok(a);
#define TB_X(w, d)                                                                                  \
  if (a.pl.W == w && a.pl.D == d) {                                                                 \
    constexpr size_t lds = ct::SlabPlan<w, d>::LDS_BYTES;                                           \
    if (r16 && raw16_early()) return launch_ct(k_slab_fwd_ct16<w, d, 768, true>, 768, lds, units, ncu, a, st); \
    if (r16) return launch_ct(k_slab_fwd_ct16<w, d, 768, false>, 768, lds, units, ncu, a, st);     \
    if (ct::SlabPlan<w, d>::FUSED_DU && (ct_fuse() & 1))                                         \
      return launch_ct(k_slab_fwd_ct<w, d, 512, true>, 512, lds, units, ncu, a, st);                \
    if (ct_nt() == 512) return launch_ct(k_slab_fwd_ct<w, d, 512, false>, 512, lds, units, ncu, a, st); \
    return launch_ct(k_slab_fwd_ct<w, d, 768, false>, 768, lds, units, ncu, a, st);                 \
  }
  TB_CT_SLAB_SHAPES(TB_X)
#undef TB_X
  return hipErrorInvalidValue;
}

hipError_t launch_slab_inv_ct(const SlabInvArgs& a, int ncu, hipStream_t st) {
  const int units = a.pl.H * a.nbc;
#define TB_X(w, d)                                                                                  \
  if (a.pl.W == w && a.pl.D == d) {                                                                 \
    constexpr size_t lds = ct::SlabPlan<w, d>::LDS_BYTES;                                           \
    if (ct::SlabPlan<w, d>::FUSED_DU && (ct_fuse() & 2))                                         \
      return launch_ct(k_slab_inv_ct<w, d, 512, true>, 512, lds, units, ncu, a, st);                \
    if (ct_nt() == 512) return launch_ct(k_slab_inv_ct<w, d, 512, false>, 512, lds, units, ncu, a, st); \
    return launch_ct(k_slab_inv_ct<w, d, 768, false>, 768, lds, units, ncu, a, st);                 \
  }
  TB_CT_SLAB_SHAPES(TB_X)
#undef TB_X
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------- half units
bool slab_half_supported(int W, int D) {
#define TB_X(w, d) if (W == w && D == d) return true;
  TB_CT_HALF_SHAPES(TB_X)
#undef TB_X
  return false;
}

// half-unit configurations (passes A / C): 0 = 256 threads with the fused DU / RE phase, 1 = 256 threads
// unfused, 2 = 512 threads unfused, 3 = 768 threads unfused.  Measured on the gibbs-aug C3 chain
// (A / C us): 0: 220 / 207, 1: 224 / 211, 2: 184 / 167, 3: 224 / 151 -> A 2, C 3.
static int half_cfg() { return 2; }
static int half_cfg_inv() { return 3; }

template <class K, class A>
static hipError_t launch_half(K kern, int nt, size_t lds, int units, const A& a, hipStream_t st) {
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(half_grid(units)), dim3(nt), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_slab_fwd_half(const SlabFwdArgs& a, hipStream_t st) {
  const int units = a.pl.H * a.nbc;
#define TB_X(w, d)                                                                                   \
  if (a.pl.W == w && a.pl.D == d) {                                                                  \
    constexpr size_t lds = ct::HalfPlan<w, d>::LDS_BYTES;                                            \
    if (half_cfg() == 3) return launch_half(k_slab_fwd_half<w, d, 768, false>, 768, lds, units, a, st); \
    if (half_cfg() == 2) return launch_half(k_slab_fwd_half<w, d, 512, false>, 512, lds, units, a, st); \
    if (half_cfg() == 1) return launch_half(k_slab_fwd_half<w, d, 256, false>, 256, lds, units, a, st); \
    return launch_half(k_slab_fwd_half<w, d, 256, true>, 256, lds, units, a, st);                    \
  }
  TB_CT_HALF_SHAPES(TB_X)
#undef TB_X
  return hipErrorInvalidValue;
}

hipError_t launch_slab_inv_half(const SlabInvArgs& a, hipStream_t st) {
  const int units = a.pl.H * a.nbc;
#define TB_X(w, d)                                                                                   \
  if (a.pl.W == w && a.pl.D == d) {                                                                  \
    constexpr size_t lds = ct::HalfPlan<w, d>::LDS_BYTES;                                            \
    if (half_cfg_inv() == 3) return launch_half(k_slab_inv_half<w, d, 768, false>, 768, lds, units, a, st); \
    if (half_cfg_inv() == 2) return launch_half(k_slab_inv_half<w, d, 512, false>, 512, lds, units, a, st); \
    if (half_cfg_inv() == 1) return launch_half(k_slab_inv_half<w, d, 256, false>, 256, lds, units, a, st); \
    return launch_half(k_slab_inv_half<w, d, 256, true>, 256, lds, units, a, st);                    \
  }
  TB_CT_HALF_SHAPES(TB_X)
#undef TB_X
  return hipErrorInvalidValue;
}

}  // namespace tb
