// kern_band.hip -- the band-limited k-space passes A' / B' / C' (band.h) and the identity copy.
//
// Reference restated (file:line under /root/reference):
//   Fourier.shift_fourier / inv_shift_fourier     source_code/filters_and_operators.py:594-632
//   RandFourierDiskMaskd (low-pass disk)           source_code/filters_and_operators.py:236-279
//   RandPlaneWaves_ellipsoid / KSpaceSpikeNoise    :370-414 / :906-983 (point updates)
//   WrapArtifact, GibbsNoise, GibbsNoiseLayer      :503-515, :678-705, stylization_layers.py:91-116
// The op program is applied by apply_ops (fft_core.h), shared with the full-spectrum pass B.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

#include "band.h"

namespace tb {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// row of register s of a 32x32 MFMA accumulator (lane half 0; +4 for lanes 32-63)
__device__ __forceinline__ int acc_row(int s) { return (s & 3) + 8 * (s >> 2); }  // rho(s)

__device__ __forceinline__ float2 ld2(const cf* p) {
  const cf v = *p;
  return make_float2(v.x, v.y);
}

// ----------------------------------------------------------------------------- pass A'
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

// x = h + l with h = f16(x), l = f16(x - h): 22 significant bits (|x| < 2^15 after scaling)
__device__ __forceinline__ void split_f16(float x, _Float16& h, _Float16& l) {
  h = (_Float16)x;
  l = (_Float16)(x - (float)h);
}

// Global -> LDS copy of n elements of T by the whole workgroup with U loads in flight per thread
// (a plain loop would wait for every load before its LDS store: one memory round trip per
// iteration, ~20 of them in a kernel prologue before the first output is written).
template <int U, class T>
__device__ __forceinline__ void lds_fill(T* dst, const T* __restrict__ src, int n, int tid) {
  for (int base = 0; base < n; base += U * BAND_NT) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // clamped index: every lane loads, no divergent partial array
      const int i = base + u * BAND_NT + tid;
      v[u] = src[i < n ? i : n - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * BAND_NT + tid;
      if (i < n) dst[i] = v[u];
    }
  }
}

constexpr int FWD_PF = 10;  // 16-B prefetch registers per lane: a 16-row strip of D <= 159

// One strip (<= 16 rows of a slab): where it starts and how it sits in memory.
struct StripSrc {
  const float* src;  // first element of the strip's first row
  int nr;            // rows
  int total;         // rows * D
  int off;           // src - (16-B aligned start), in floats
  int nq;            // 16-B vectors covering the strip (contiguous rows)
};

// Wave-private strip staging.  The wave's 64 lanes issue the strip's 16-B loads into registers
// (FWD_PF per lane) one strip ahead, then store them to the wave's LDS region:
//   odd D   -- pitch D, the strip is one contiguous run in LDS as in memory; element e sits at
//              Xw[off + e], so every 16-B vector lands 16-B aligned (ds_write_b128);
//   D % 4 == 0, compiled D, aligned rows -- pitch D + 4: a vector never straddles a row, one
//              ds_write_b128 at e + 4 (e / D);
//   other even D -- pitch D + 1, element-wise.
template <int DC>
struct Strip {
  __device__ __forceinline__ static void load(f32x4 (&v)[FWD_PF], const StripSrc& s, int lane) {
    const f32x4* s4 = reinterpret_cast<const f32x4*>(s.src - s.off);
#pragma unroll
    for (int u = 0; u < FWD_PF; ++u) {
      const int q = lane + 64 * u;
      if (q < s.nq) v[u] = __builtin_nontemporal_load(s4 + q);
    }
  }
  // returns the strip's row-0 pointer in LDS
  __device__ __forceinline__ static const float* store(float* Xw, const f32x4 (&v)[FWD_PF], const StripSrc& s, int D,
                                                      int P, const FastDiv& fd, int lane) {
    if (D & 1) {
#pragma unroll
      for (int u = 0; u < FWD_PF; ++u) {
        const int q = lane + 64 * u;
        if (q < s.nq) *reinterpret_cast<f32x4*>(Xw + 4 * q) = v[u];
      }
      return Xw + s.off;
    }
    if (DC > 0 && P == D + 4) {  // off == 0 (host-checked alignment)
#pragma unroll
      for (int u = 0; u < FWD_PF; ++u) {
        const int q = lane + 64 * u;
        if (q < s.nq) *reinterpret_cast<f32x4*>(Xw + 4 * q + 4 * ((4 * q) / D)) = v[u];
      }
      return Xw;
    }
#pragma unroll
    for (int u = 0; u < FWD_PF; ++u) {
      const int e0 = 4 * (lane + 64 * u) - s.off;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = e0 + k;
        if (e >= 0 && e < s.total) Xw[e + fd.div(e)] = v[u][k];
      }
    }
    return Xw;
  }
};
// strided rows or a long D (e.g. the padded U-Net buffer filtered in place): plain copy by the wave
__device__ __forceinline__ void strip_copy(float* Xw, int P, const StripSrc& s, int64_t sw, int D, const FastDiv& fd,
                                           int lane) {
  for (int e0 = lane; e0 < s.total; e0 += 8 * 64) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = e0 + k * 64;
      if (e < s.total) {
        const int r = fd.div(e);
        v[k] = s.src[(int64_t)r * sw + (e - r * D)];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = e0 + k * 64;
      if (e < s.total) {
        const int r = fd.div(e);
        Xw[r * P + (e - r * D)] = v[k];
      }
    }
  }
}

// NT2: 16-wide kd tiles (NDk <= 16 NT2); KWT: 16-wide kw tiles (KW < 16 KWT); DC: compiled D
// (0: runtime D, D-product table read from LDS).  Per 16-row strip, on the wave alone:
//   D product  R(row, kd) = sum_d s_d cos + i sum_d t_d sin      16x16x4 MFMA, folded over (d, D-d)
//   W product  O(kw, kd) += sum_rows {cos, sin}(2 pi kw w / W) R  16x16x4 MFMA; the B operand is the
//              D product's accumulator register j (its rows 4 (l/16) + j are the k index), so R never
//              leaves the registers.
// At the end of the wave's part of a slab, O goes through the wave's LDS region into the slab's
// partial-sum slot P[bc][h][seg] (seg = this wave's rank among the slab's waves).
// F16 (compiled D, NT2 = 1, 16-B staged strips): the D product in split f16 on mfma_f32_16x16x32_f16 --
// per strip the folded values s, t scaled by a power of two from the strip's max |x| (|s|, |t| < 2^15),
// split into f16 pairs, three products (sh Th + sh Tl + sl Th) against the plan's split table (x 2^8),
// 32 folded d per k-step: 18 MFMAs of 16 cycles per strip instead of 40 of 32 (f32 16x16x4).  The
// scale is undone in the W product's A operand (cos, sin x 2^-(8 + scale exponent), exact).
template <int NT2, int KWT, int DC, bool F16 = false>
__global__ __launch_bounds__(BAND_NT) __attribute__((amdgpu_waves_per_eu(NT2 * KWT == 1 ? 3 : NT2 * KWT == 2 ? 2 : 1, 4))) void k_band_fwd(BandFwdArgs) {
  static_assert(!F16 || (DC > 0 && NT2 == 1), "split-f16 D product: compiled D, one kd tile");
  const BandFwdArgs& a = kargs<BandFwdArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W;
  const int D = DC > 0 ? DC : a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, ncol = a.g.ncol;
  const int P = band_fwd_pitch(D, DC > 0);
  const int Ld = D / 2 + 1;                 // folded d in [0, D/2]
  const int KSd = (Ld + 3) / 4;             // 16x16x4 k-steps of the D product
  constexpr int KSC = DC > 0 ? (DC / 2 + 1 + 3) / 4 : 1;
  const int XW = band_fwd_xw(P, NT2, KWT);
  float2* twW = reinterpret_cast<float2*>(smem);                               // (cos, -sin)(2 pi t / W)
  // (F16: no W twiddles in LDS -- read per strip from the plan, which keeps three workgroups per CU)
  float* Bt = reinterpret_cast<float*>(smem + (F16 ? 0 : ((W * 8 + 15) & ~15)));  // [NT2][KSd][2][64] (DC == 0)
  constexpr int KS16 = DC > 0 ? band_fwd16_ks(DC) : 1;
  // F16: the split-f16 D-product B fragments [k-step][cos/sin][hi/lo][64 lanes] (16 B each) in the Bt region
  float* Xw = Bt + (F16 ? KS16 * 4 * 64 * 4 : DC > 0 ? 0 : NT2 * KSd * 128) + wv * XW;  // this wave's region
  const h16x8* T16s = reinterpret_cast<const h16x8*>(Bt);
  const FastDiv fd = FastDiv::make(D);
  const FwdSplit sp = a.split;
  const uint32_t nst = sp.nst;
  const uint32_t gw = (uint32_t)blockIdx.x * 4 + (uint32_t)wv;
  uint32_t t = 0, t1 = 0;
  if (gw < sp.G) {
    t = fwd_start(sp, gw);
    t1 = fwd_start(sp, gw + 1);
  }
  const bool pre = F16 || (a.vec && (BAND_FWD_ROWS * D + 6) <= 4 * 64 * FWD_PF);  // F16: host-checked
  const int diag = a.diag;
  auto strip_src = [&](uint32_t tt) {
    StripSrc s;
    const uint32_t slab = tt / nst, st = tt - slab * nst;
    const uint32_t bcl = slab / (uint32_t)H, h = slab - bcl * (uint32_t)H;
    const int w0 = (int)st * BAND_FWD_ROWS;
    s.src = a.x + (int64_t)(a.bc0 + (int)bcl) * a.sbc + (int64_t)h * a.sh + (int64_t)w0 * a.sw;
    s.nr = (W - w0) < BAND_FWD_ROWS ? (W - w0) : BAND_FWD_ROWS;
    s.total = s.nr * D;
    s.off = (int)((reinterpret_cast<uintptr_t>(s.src) >> 2) & 3);
    s.nq = (s.total + s.off + 3) >> 2;
    return s;
  };
  // the first strip's loads fly while the tables fill
  f32x4 pf[FWD_PF];
  StripSrc ss{};
  if (t < t1) {
    ss = strip_src(t);
    if (pre) Strip<DC>::load(pf, ss, lane);
  }
  float btr[F16 ? 1 : NT2][F16 ? 1 : KSC][2];  // compiled D: the D-product B fragments live in registers
  if constexpr (DC > 0 && !F16) {
#pragma unroll
    for (int nt = 0; nt < NT2; ++nt)
#pragma unroll
      for (int k = 0; k < KSC; ++k) {
        btr[nt][k][0] = a.tbt[((nt * KSC + k) * 2) * 64 + lane];
        btr[nt][k][1] = a.tbt[((nt * KSC + k) * 2 + 1) * 64 + lane];
      }
  }
  if (!F16) lds_fill<4>(twW, reinterpret_cast<const float2*>(a.pl.tw[1]), W, tid);
  // plan table (host double precision); 8-B pieces
  if (DC == 0) lds_fill<8>(reinterpret_cast<float2*>(Bt), reinterpret_cast<const float2*>(a.tbt), NT2 * KSd * 64, tid);
  if (F16) lds_fill<3>(reinterpret_cast<float4*>(Bt), reinterpret_cast<const float4*>(a.tbt16), KS16 * 4 * 64, tid);
  __syncthreads();  // the only workgroup barrier: tables in LDS
  if (t >= t1) return;
  // O accumulators: [cos/sin][re/im][kw tile][kd tile]
  f32x4 oacc[2][2][KWT][NT2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int kt = 0; kt < KWT; ++kt)
#pragma unroll
        for (int nt = 0; nt < NT2; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) oacc[m][r][kt][nt][j] = 0.f;
  for (;;) {
    const uint32_t slab = t / nst, st = t - slab * nst;
    const int w0 = (int)st * BAND_FWD_ROWS, nr = ss.nr;
    // 1. this strip into the wave's LDS region (F16: and its scale from max |x| of the loaded vectors)
    float wsc = 1.f;  // F16: the W product's twiddle factor 2^-(8 + e)
    float ssc = 1.f;  // F16: the strip's scale 2^(14 - e), max |x| < 2^e
    float2 twr[F16 ? KWT : 1][4];  // F16: this strip's W twiddles, loaded before the next strip's vectors
    if (F16) {
      const int wl = w0 + 4 * l4;
#pragma unroll
      for (int kt = 0; kt < KWT; ++kt) {
        const int kw = 16 * kt + l15;
        int tw = (int)(((int64_t)kw * wl) % W);
        const int step = kw % W;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          twr[kt][j] = reinterpret_cast<const float2*>(a.pl.tw[1])[tw];
          tw += step;
          tw = tw >= W ? tw - W : tw;
        }
      }
      float mx = 0.f;
#pragma unroll
      for (int u = 0; u < FWD_PF; ++u) {  // branch-free: vectors past the strip count as 0
        const float m4 = fmaxf(fmaxf(fabsf(pf[u][0]), fabsf(pf[u][1])), fmaxf(fabsf(pf[u][2]), fabsf(pf[u][3])));
        mx = fmaxf(mx, lane + 64 * u < ss.nq ? m4 : 0.f);
      }
      mx = wave_max(mx);
      int ex;
      (void)frexpf(mx, &ex);  // mx < 2^ex (0 for a zero strip)
      ssc = ldexpf(1.f, 14 - ex);
      wsc = ldexpf(1.f, ex - 14) * (1.f / BAND_FWD16_TSCALE);
    }
    const float* xs = Xw;
    if (diag & 2)
      xs = Xw;
    else if (pre)
      xs = Strip<DC>::store(Xw, pf, ss, D, P, fd, lane);
    else
      strip_copy(Xw, P, ss, a.sw, D, fd, lane);
    if (nr < BAND_FWD_ROWS) {  // a short last strip: the rows past W read as zeros (weight 0 below)
      float* z = const_cast<float*>(xs) + nr * P;
      for (int i = lane; i < (BAND_FWD_ROWS - nr) * P; i += 64) z[i] = 0.f;
    }
    __builtin_amdgcn_wave_barrier();
    // 2. the next strip's loads fly while this one is computed
    const uint32_t tn = t + 1;
    if (tn < t1) {
      ss = strip_src(tn);
      if (pre && !(diag & 1)) Strip<DC>::load(pf, ss, lane);
    }
    // 3. D product
    f32x4 accc[NT2], accs[NT2];
#pragma unroll
    for (int nt = 0; nt < NT2; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) accc[nt][j] = accs[nt][j] = 0.f;
    if (!(diag & 4)) {
      const float* row = xs + l15 * P;
      if constexpr (F16) {  // lane (row l15, quarter l4): folded d = 32 k + 8 l4 + i of its row
#pragma unroll
        for (int k = 0; k < KS16; ++k) {
          h16x8 sh, sl, th, tl;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int d = 32 * k + 8 * l4 + i;  // < 96 <= D - 32: both reads inside the row
            const bool has = d < Ld;
            const bool pair = d >= 1 && 2 * d < D;
            const float xa = has ? row[d] : 0.f;
            const float xm = pair ? row[D - d] : 0.f;
            _Float16 a0, a1, b0, b1;
            split_f16((xa + xm) * ssc, a0, a1);
            split_f16(pair ? (xm - xa) * ssc : 0.f, b0, b1);
            sh[i] = a0;
            sl[i] = a1;
            th[i] = b0;
            tl[i] = b1;
          }
          const h16x8* tk = T16s + (k * 4) * 64 + lane;  // [cos hi, cos lo, sin hi, sin lo]
          const h16x8 ch = tk[0], cl = tk[64], sh2 = tk[128], sl2 = tk[192];
          accc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(sh, ch, accc[0], 0, 0, 0);
          accs[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(th, sh2, accs[0], 0, 0, 0);
          accc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(sh, cl, accc[0], 0, 0, 0);
          accs[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(th, sl2, accs[0], 0, 0, 0);
          accc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(sl, ch, accc[0], 0, 0, 0);
          accs[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(tl, sh2, accs[0], 0, 0, 0);
        }
      } else if (DC > 0) {
#pragma unroll
        for (int k = 0; k < KSC; ++k) {
          const int d = 4 * k + l4;
          const bool has = d < Ld;
          const bool pair = d >= 1 && 2 * d < D;
          const float xa = has ? row[d] : 0.f;
          const float xm = pair ? row[D - d] : 0.f;
          const float sv = xa + xm, tv = pair ? xm - xa : 0.f;
#pragma unroll
          for (int nt = 0; nt < NT2; ++nt) {
            accc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(sv, btr[nt][k][0], accc[nt], 0, 0, 0);
            accs[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(tv, btr[nt][k][1], accs[nt], 0, 0, 0);
          }
        }
      } else {
        for (int k0 = 0; k0 < KSd; k0 += 4) {
          float sv[4], tv[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // all LDS reads of 4 k-steps first
            const int d = 4 * (k0 + q) + l4;
            const bool has = d < Ld;
            const bool pair = d >= 1 && 2 * d < D;
            const float xa = has ? row[d] : 0.f;
            const float xm = pair ? row[D - d] : 0.f;
            sv[q] = xa + xm;
            tv[q] = pair ? xm - xa : 0.f;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (k0 + q >= KSd) break;
#pragma unroll
            for (int nt = 0; nt < NT2; ++nt) {
              const float* bt = Bt + ((nt * KSd + k0 + q) * 2) * 64 + lane;
              accc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(sv[q], bt[0], accc[nt], 0, 0, 0);
              accs[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(tv[q], bt[64], accs[nt], 0, 0, 0);
            }
          }
        }
      }
    }
    // 4. W product: rows w = w0 + 4 (l/16) + j of the strip; rows >= W weigh 0
    if (!(diag & 8)) {
      const int wl = w0 + 4 * l4;
#pragma unroll
      for (int kt = 0; kt < KWT; ++kt) {
        const int kw = 16 * kt + l15;
        int tw = (int)(((int64_t)kw * wl) % W);
        const int step = kw % W;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = wl + j < W && kw <= KW;
          const float2 c = F16 ? twr[F16 ? kt : 0][j] : twW[tw];
          const float ca = ok ? c.x * wsc : 0.f, sa = ok ? -c.y * wsc : 0.f;
#pragma unroll
          for (int nt = 0; nt < NT2; ++nt) {
            oacc[0][0][kt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca, accc[nt][j], oacc[0][0][kt][nt], 0, 0, 0);
            oacc[0][1][kt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca, accs[nt][j], oacc[0][1][kt][nt], 0, 0, 0);
            oacc[1][0][kt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(sa, accc[nt][j], oacc[1][0][kt][nt], 0, 0, 0);
            oacc[1][1][kt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(sa, accs[nt][j], oacc[1][1][kt][nt], 0, 0, 0);
          }
          tw += step;
          tw = tw >= W ? tw - W : tw;
        }
      }
    }
    // 5. end of this wave's part of the slab: O -> LDS region -> the slab's partial-sum slot
    if (st == nst - 1 || tn == t1) {
      float* Ob = Xw;  // [m][r][kt][nt][64 lanes][4]; the strip is consumed (LDS ops stay in order)
      constexpr int NB = 2 * 2 * KWT * NT2;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int kt = 0; kt < KWT; ++kt)
#pragma unroll
            for (int nt = 0; nt < NT2; ++nt) {
              const int blk = ((m * 2 + r) * KWT + kt) * NT2 + nt;
              *reinterpret_cast<f32x4*>(Ob + (blk * 64 + lane) * 4) = oacc[m][r][kt][nt];
              oacc[m][r][kt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
      __builtin_amdgcn_wave_barrier();
      const int seg = (int)(gw - fwd_wave_of(sp, slab * nst));
      const int bcl = (int)(slab / (uint32_t)H), h = (int)(slab - (uint32_t)bcl * (uint32_t)H);
      cf* Pb = a.P + (((int64_t)(a.bc0 + bcl) * H + h) * BAND_FWD_SEGS + seg) * ncol;
      for (int it = lane; it < (KW + 1) * NDk; it += 64) {
        const int kw = it / NDk, kd = it - kw * NDk;
        const int kt = kw >> 4, nt = kd >> 4;
        // C layout: lane = 16 (row / 4) + col, register = row % 4 (row = kw % 16, col = kd % 16)
        const int ln = 16 * ((kw & 15) >> 2) + (kd & 15), rg = kw & 3;
        float o[2][2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 2; ++r) o[m][r] = Ob[((((m * 2 + r) * KWT + kt) * NT2 + nt) * 64 + ln) * 4 + rg];
        // P(kw) = Ac - i As, P(-kw) = Ac + i As
        Pb[(KW + kw) * NDk + kd] = mk(o[0][0] + o[1][1], o[0][1] - o[1][0]);
        if (kw > 0) Pb[(KW - kw) * NDk + kd] = mk(o[0][0] - o[1][1], o[0][1] + o[1][0]);
      }
      (void)NB;
      __builtin_amdgcn_wave_barrier();
    }
    if (tn >= t1) break;
    t = tn;
  }
}

// ----------------------------------------------------------------------------- pass B'
// One workgroup (2 waves) per (bc, 16 box columns); the H transforms are f32 MFMA products
// (v_mfma_f32_32x32x2f32: exact f32 products and sums):
//   stage    the columns' pass-A' partial sums for every slab, segments added, into LDS (each
//            partial sum read once, ~30 loads in flight per lane);
//   forward  [C; S](kh, h) . [P.re P.im](h, col) over h -- rows 16 kh cosines then their 16 sines
//            per 32-row tile, columns (col, re/im); the waves take a quarter of h each (operands of
//            6 steps read from LDS ahead of their MFMAs) and meet in LDS: (Ac.re, Ac.im, As.re,
//            As.im) = the sums of pass B;
//   program  the sample's op program (apply_ops, the code of pass B) on Q(kh) = Ac - i As and
//            Q(-kh) = Ac + i As, kept as G rows (A.re, A.im | -B.im, B.re), A / B = Q'(kh) +/- Q'(-kh);
//   inverse  Z(h, col) = [cos sin](h, (kh, t)) . G((kh, t), col) per 32-slab tile, the tiles dealt
//            to the waves, written over the slab's first partial-sum slot (own columns only).
constexpr int BAND_HC_CB = 16;  // box columns per workgroup
template <int MT>               // 32-row tiles of [C; S]: KH + 1 <= 16 MT
__global__ __launch_bounds__(64 * BAND_HC_NW) void k_band_hcol(BandMidArgs) {
  const BandMidArgs& a = kargs<BandMidArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63, hl = lane >> 5, l31 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, KH = a.g.KH, ncol = a.g.ncol;
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int c0 = (int)blockIdx.x * BAND_HC_CB;
  float2* Pb = reinterpret_cast<float2*>(smem);                     // [H + 1][16] (row H: zeros)
  float2* tw = Pb + (size_t)(H + 1) * BAND_HC_CB;                   // (cos, -sin)(2 pi t / H)
  float* Qs = reinterpret_cast<float*>(tw + H);                     // [MT][32][32]
  float* G = Qs + MT * 1024;                                        // [2 (KH + 1)][32]
  cf* P = a.P + (int64_t)bc * H * BAND_FWD_SEGS * ncol;
  constexpr int NT = 64 * BAND_HC_NW;
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0 && a.cnt) *a.cnt = 0u;
  if (blockIdx.x == 0 && blockIdx.y == 0 && a.mm && tid < 2 * (a.nbc / a.C))  // pass C''s key atomics start here
    a.mm[2 * (a.bc0 / a.C) + tid] = (tid & 1) ? 0u : 0xffffffffu;
  for (int hh = tid; hh < H; hh += NT) tw[hh] = ld2(a.pl.tw[0] + hh);
  if (tid < BAND_HC_CB) Pb[H * BAND_HC_CB + tid] = make_float2(0.f, 0.f);
  {  // stage: lane -> (h offset tid >> 4, column tid & 15); UR slab rows x 3 slots in flight
    const int c = tid & 15, col = c0 + c;
    const bool ok = col < ncol;
    constexpr int UR = 8, RS = NT / 16;
    for (int hb = tid >> 4; hb < H; hb += RS * UR) {
      float2 v[UR][3];
      int ns[UR];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int hh = hb + RS * u < H ? hb + RS * u : H - 1;
        ns[u] = (ok && hb + RS * u < H) ? fwd_nseg(a.split, (uint32_t)(bcl * H + hh)) : 0;
        const cf* ph = P + (int64_t)hh * BAND_FWD_SEGS * ncol + (ok ? col : 0);
#pragma unroll
        for (int sg = 0; sg < 3; ++sg) v[u][sg] = ld2(ph + sg * ncol);
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        if (hb + RS * u >= H) break;
        float2 z = make_float2(0.f, 0.f);
#pragma unroll
        for (int sg = 0; sg < 3; ++sg) {
          z.x += sg < ns[u] ? v[u][sg].x : 0.f;
          z.y += sg < ns[u] ? v[u][sg].y : 0.f;
        }
        Pb[(hb + RS * u) * BAND_HC_CB + c] = z;
      }
    }
  }
  __syncthreads();
  // forward: this wave's quarter of the h pairs, 6 steps' operands read ahead of their MFMAs
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[mt][j] = 0.f;
  {
    const int nst = (H + 1) / 2, sh = (nst + BAND_HC_NW - 1) / BAND_HC_NW;
    const int s0 = wv * sh, s1 = s0 + sh < nst ? s0 + sh : nst;
    const int bcol = l31 >> 1, bcomp = l31 & 1;
    int tA[MT], dA[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int kh = 16 * mt + (l31 & 15);
      tA[mt] = (int)(((int64_t)kh * (2 * s0 + hl)) % H);
      dA[mt] = (2 * kh) % H;
    }
    constexpr int US = 6;
    for (int st = s0; st < s1; st += US) {
      float bv[US], av[US][MT];
#pragma unroll
      for (int u = 0; u < US; ++u) {
        const int h = 2 * (st + u) + hl;  // past this wave's steps / h == H: the zero row
        const float2 pv = Pb[(st + u < s1 && h < H ? h : H) * BAND_HC_CB + bcol];
        bv[u] = bcomp ? pv.y : pv.x;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const float2 w = tw[tA[mt]];
          av[u][mt] = (l31 < 16) ? w.x : -w.y;  // cos rows, then sin rows
          tA[mt] += dA[mt];
          tA[mt] = tA[mt] >= H ? tA[mt] - H : tA[mt];
        }
      }
#pragma unroll
      for (int u = 0; u < US; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][mt], bv[u], acc[mt], 0, 0, 0);
    }
  }
  // the waves' sums meet in LDS: [wave][MT 32 x 32], then summed per element
  float* red = G + 2 * (KH + 1) * 32;  // [NW][MT][32][32]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((wv * MT + mt) * 32 + acc_row(r) + 4 * hl) * 32 + l31] = acc[mt][r];
  __syncthreads();
  for (int e = tid; e < MT * 1024; e += NT) {
    float q = red[e];
#pragma unroll
    for (int w_ = 1; w_ < BAND_HC_NW; ++w_) q += red[w_ * MT * 1024 + e];
    Qs[e] = q;
  }
  __syncthreads();
  const int lb = a.cofs + bcl, s = lb / a.C, chan = lb - s * a.C;
  const tb_sample_ops& so = a.ops.s[s];
  for (int it = tid; it < (KH + 1) * BAND_HC_CB; it += NT) {  // the op program, once per (kh, column)
    const int k = it / BAND_HC_CB, c = it - k * BAND_HC_CB, cl = c0 + c;
    const float* q = Qs + (k >> 4) * 1024 + (k & 15) * 32 + 2 * c;  // C rows; S rows 16 below
    const float acr = q[0], aci = q[1], asr = q[512], asi = q[513];
    float4 ab = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cl < ncol) {
      const int jw = cl / NDk, kd = cl - jw * NDk;
      const FreqCol fc = freq_col((jw - KW + W) % W, kd, W, D);
      const cf qp = apply_ops(so, chan, mk(acr + asi, aci - asr), fc, k, H);
      const cf qm = k == 0 ? mk(0.f, 0.f) : apply_ops(so, chan, mk(acr - asi, aci + asr), fc, H - k, H);
      ab = k == 0 ? make_float4(qp.x, qp.y, 0.f, 0.f) : make_float4(qp.x + qm.x, qp.y + qm.y, qp.x - qm.x, qp.y - qm.y);
    }
    G[(2 * k) * 32 + 2 * c] = ab.x;           // cos row: (A.re, A.im)
    G[(2 * k) * 32 + 2 * c + 1] = ab.y;
    G[(2 * k + 1) * 32 + 2 * c] = -ab.w;      // sin row: (-B.im, B.re)
    G[(2 * k + 1) * 32 + 2 * c + 1] = ab.z;
  }
  __syncthreads();
  // inverse: 32-slab tiles dealt to the waves, 4 steps' operands read ahead of their MFMAs
  float* Pf = reinterpret_cast<float*>(P);
  const int col = c0 + (l31 >> 1);
  for (int ht = wv; ht * 32 < H; ht += BAND_HC_NW) {
    f32x16 z;
#pragma unroll
    for (int j = 0; j < 16; ++j) z[j] = 0.f;
    const int h = 32 * ht + l31;
    const int hm = h < H ? h : 0;
    int t = 0;
    for (int k0 = 0; k0 <= KH; k0 += 4) {
      float av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = k0 + u <= KH;
        const float2 w = tw[t];
        av[u] = ok ? (hl ? -w.y : w.x) : 0.f;  // k-slot (k, cos) on lanes 0-31, (k, sin) on 32-63
        bv[u] = ok ? G[(2 * (k0 + u) + hl) * 32 + l31] : 0.f;
        t += hm;
        t = t >= H ? t - H : t;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], z, 0, 0, 0);
    }
    if (col < ncol)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int hh = 32 * ht + acc_row(r) + 4 * hl;
        if (hh < H) Pf[((int64_t)hh * BAND_FWD_SEGS * ncol + col) * 2 + (l31 & 1)] = z[r];
      }
  }
  // the out-of-box spike points: the program applied to a coefficient the low-pass zeroed
  if (blockIdx.x == 0 && tid < BAND_MAX_PTS) {
    const BandSamplePts& sp = a.sp[s];
    cf c = mk(0.f, 0.f);
    if (tid < sp.n) {
      const BandPt pt = sp.p[tid];
      c = apply_ops(so, chan, mk(0.f, 0.f), freq_col(pt.kw, pt.kd, W, D), pt.kh, H);
    }
    a.pts[(int64_t)bc * BAND_MAX_PTS + tid] = c;
  }
}

// ----------------------------------------------------------------------------- pass B2'
__device__ void band_tab16(const BandMidArgs& a, int t);  // pass C''s split-f16 table (below)
// Z_h(col) = A_0 + sum_kh>=1 (A cos + i B sin), theta = 2 pi kh h / H, for every slab h: lanes =
// columns (AB loaded once per lane), waves = slabs (twiddles wave-uniform).  Written over P.
__global__ __launch_bounds__(BAND_NT) void k_band_zh(BandMidArgs) {
  // One slab (bc, h) per wave: Z_h(col) = A_0 + sum_kh>=1 (A cos + i B sin), then the slab's
  // V-product matrix M2T(v, k) written in MFMA A-fragment order [vt][ks][64 lanes], so that pass C'
  // loads each k-step's fragment as one coalesced 256-B read:
  //   rows v = 2 kd + (re, im): Vr = sum_kw (Ar cos - Bi sin), Vi = sum_kw (Ai cos + Br sin),
  //     A/B = Z(kw) +/- Z(-kw), scaled by the C2R weight wt(kd) / N;
  //   rows 2 (NDk + j) + (re, im): the out-of-box point j, ph_j = c_j e^{+2 pi i kh_j h / H} wt / N,
  //     on its own k-step KW + 1 + j.
  const BandMidArgs& a = kargs<BandMidArgs>();
  __shared__ float2 zs[4][BAND_MAX_ZCOL];
  __shared__ float2 phs[4][BAND_MAX_PTS];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, D = a.pl.D, KH = a.g.KH, KW = a.g.KW, NDk = a.g.NDk, ncol = a.g.ncol;
  const int npm = a.g.KS - NDk, KV = KW + 1 + npm, VT = band_vt(a.g);
  const int nzb = (H * a.nbc + 3) / 4;  // blocks past these build the split-f16 synthesis table
  if ((int)blockIdx.x >= nzb) {
    band_tab16(a, ((int)blockIdx.x - nzb) * BAND_NT + tid);
    return;
  }
  const int u = (int)blockIdx.x * 4 + wv;
  if (u >= H * a.nbc) return;
  const int bcl = u / H, h = u - bcl * H, bc = a.bc0 + bcl;
  const int s = (a.cofs + bcl) / a.C;
  (void)KH;
  const cf* Zr = a.P + ((int64_t)bc * H + h) * BAND_FWD_SEGS * ncol;  // Z_h (pass B', first slot)
  for (int col = lane; col < ncol; col += 64) zs[wv][col] = ld2(Zr + col);
  const BandSamplePts& sp = a.sp[s];
  if (lane < BAND_MAX_PTS) {
    float2 v = make_float2(0.f, 0.f);
    if (lane < sp.n && lane < npm) {
      const cf c = a.pts[(int64_t)bc * BAND_MAX_PTS + lane];
      const cf tw = a.pl.tw[0][(int)(((int64_t)sp.p[lane].kh * h) % H)];
      const float wt = ((sp.p[lane].kd == 0 || 2 * sp.p[lane].kd == D) ? 1.f : 2.f) * a.scale;
      v = make_float2((c.x * tw.x + c.y * tw.y) * wt, (c.y * tw.x - c.x * tw.y) * wt);
    }
    phs[wv][lane] = v;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
  const float2* Zb = zs[wv];
  const int nrv = band_rows(a.g);
  const int pbase = a.g.cat ? a.p0[s] : 0;  // g.cat: this sample's first point row pair past the band rows
  float* F = a.M2F + (int64_t)u * VT * KV * 64;
  for (int vt = 0; vt < VT; ++vt)
    for (int ks = 0; ks < KV; ++ks) {
      const int r = 32 * vt + (lane & 31), sn = lane >> 5;
      const int im = r & 1, kd = r >> 1;
      float v = 0.f;
      if (r < nrv) {
        if (kd < NDk) {
          if (ks <= KW) {
            const float2 zp = Zb[(KW + ks) * NDk + kd];
            const float2 zm = ks > 0 ? Zb[(KW - ks) * NDk + kd] : make_float2(0.f, 0.f);
            const float ax = zp.x + zm.x, ay = zp.y + zm.y;
            const float bx = ks > 0 ? zp.x - zm.x : 0.f, by = ks > 0 ? zp.y - zm.y : 0.f;
            const float wt = ((kd == 0 || 2 * kd == D) ? 1.f : 2.f) * a.scale;
            v = (im ? (sn ? bx : ay) : (sn ? -by : ax)) * wt;
          }
        } else {
          const int j = kd - NDk - pbase;  // the sample's point j (its own V-product k-step KW + 1 + j)
          if (j >= 0 && j < sp.n && ks == KW + 1 + j) {
            const float2 c = phs[wv][j];
            v = im ? (sn ? c.x : c.y) : (sn ? -c.y : c.x);
          }
        }
      }
      F[((int64_t)vt * KV + ks) * 64 + lane] = v;
    }
}

// ----------------------------------------------------------------------------- pass C'

// Per (bc, h) slab, on the matrix cores after a small prologue:
//   V^T(v, w)  = M2T(v, k) . CS(k, w)       MFMA 32x32x2; v = 2 kd + (re, im) and two rows per
//                out-of-box point; k = (kw, cos/sin) terms and one pair per point; w on the lane
//   E(d, w)    = Bc^T(d, v_re) . V^T(v_re, w),   O(d, w) = Bs^T(d, v_im) . V^T(v_im, w)
//                MFMA with V^T straight from the accumulators: accumulator register s holds the
//                row pair (rho(s), rho(s) + 4) -- both real parts when s % 4 is even, both
//                imaginary parts when odd -- so it is the B operand of one k-step as it stands
//   y[w][d] = E - O,  y[w][D - d] = E + O   for d in [0, D/2]  (the C2R folded over d <-> D - d)
// Each lane ends with 4 consecutive columns of one image row for both halves: 16-B stores.
#ifndef TB_INV_PRIO
#define TB_INV_PRIO 2  // 2: store phases at raised wave priority (C3 -2 %, C2 -5 %); 1: MFMA phases; 0: off
#endif
#ifndef TB_INV_WPE
#define TB_INV_WPE 3  // waves per SIMD the VT = 1 kernel is compiled for (register budget)
#endif
template <int VT>  // 32-row tiles of V (2 (NDk + points) <= 32 VT)
__global__ __launch_bounds__(BAND_NT) __attribute__((amdgpu_waves_per_eu(VT == 1 ? TB_INV_WPE : 2, 4))) void k_band_inv(BandInvArgs) {
  // The workgroup takes its slabs in batches of BAND_SLOTS: the batch's inputs (V-product
  // fragments from pass B2', the samples' point rows of the synthesis table) are loaded into LDS
  // first, so that the (slab, 32-row tile) units the four waves then work through issue only
  // stores -- no load waits behind the CU's queue of outgoing image rows.
  const BandInvArgs& a = kargs<BandInvArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63, hl = lane >> 5, l31 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, NCOL = a.g.NCOL;
  const int npm = a.g.KS - NDk;        // point rows of the launch (max over its samples)
  const int KV = KW + 1 + npm;         // k-steps of the V product
  const int Dh = D / 2 + 1;            // folded output columns d in [0, D/2]
  const int nrv = 2 * (NDk + npm);     // used rows of V / the synthesis table
  const int fsz = VT * KV * 64;        // floats of one slab's fragments
  const int psz = (2 * npm + 4) * NCOL;  // floats of one slab's point rows (+4 zero rows: see E/O)
  const BandInvCarve cv = band_inv_carve(a.g, W, D);
  float* Bimg = reinterpret_cast<float*>(smem + cv.bimg);  // [2 NDk][NCOL]: even rows cos, odd rows sin
  float2* twW = reinterpret_cast<float2*>(smem + cv.tww);  // (cos, -sin)(2 pi t / W)
  float* Fs = reinterpret_cast<float*>(smem + cv.frag);    // [BAND_SLOTS][fsz]
  float* Ps = reinterpret_cast<float*>(smem + cv.prow);    // [BAND_SLOTS][psz]
  float* stg = reinterpret_cast<float*>(smem + cv.stg) + wv * 32 * BAND_STG_P;  // this wave's 32 x 32 tile
  // the batch slabs' point kw (0 past the sample's points): read from LDS in the unit loop, which
  // must hold no vector-memory load -- its s_waitcnt vmcnt would also wait out the pending stores
  int* Pkw = reinterpret_cast<int*>(smem + cv.pkw);  // [BAND_SLOTS][BAND_MAX_PTS]
  // The tables (band rows of the synthesis table, W twiddles) load in the same round as the first
  // batch's inputs: one global latency before the first unit, not three.
  const int nbi4 = 2 * NDk * NCOL / 4;           // float4s of Bimg
  const bool twv = !(W & 1) && (reinterpret_cast<uintptr_t>(a.pl.tw[1]) & 15) == 0;
  const int ntw4 = twv ? W / 2 : 0;              // float4s of twW (else filled apart, here)
  if (!twv) lds_fill<4>(twW, reinterpret_cast<const float2*>(a.pl.tw[1]), W, tid);
  const float4* Tsrc = reinterpret_cast<const float4*>(a.tds);
  const float4* Wsrc = reinterpret_cast<const float4*>(a.pl.tw[1]);
  int tb4 = nbi4 + ntw4;                         // table float4s still to load (first batch only)
  const int ntw = (W + 31) / 32;     // 32-row tiles of a slab
  const int nslab = H * a.nbc;
  const int ntn = NCOL / 32;         // 32-column tiles of the folded row
  const int ypad = a.ypad;
  const bool mal = ((D - 3) & 3) == 0;  // mirrored 4-column groups start 16-B aligned
  const int diag = a.diag;
  if (diag & 64) return;  // measurement: launch only
  // Each workgroup owns a contiguous range of (slab, row tile) units, dealt round-robin to its
  // waves, so every wave of the grid gets the same number of units (a slab-granular split left
  // half the workgroups with 3 slabs and half with 2); the range's slabs are loaded in batches of
  // up to BAND_SLOTS.
  const int nunit = nslab * ntw;
  const int per = (nunit + (int)gridDim.x - 1) / (int)gridDim.x;
  const int ub = (int)blockIdx.x * per, ue = ub + per < nunit ? ub + per : nunit;
  for (int c0 = ub; c0 < ue;) {
    const int s0 = c0 / ntw;
    const int slast = (ue - 1) / ntw;
    const int s1 = slast < s0 + BAND_SLOTS - 1 ? slast : s0 + BAND_SLOTS - 1;
    const int c1 = (s1 + 1) * ntw < ue ? (s1 + 1) * ntw : ue;  // units [c0, c1) of this batch
    const int nb = s1 - s0 + 1;
    __syncthreads();  // the previous batch is done with Fs / Ps
    {  // [tables,] the batch's fragments (contiguous slabs) and point rows: rounds of loads in flight
      const int nf4 = nb * fsz / 4, np4 = nb * psz / 4, nc4 = NCOL / 4, pp4 = psz / 4;
      const int ntot = tb4 + nf4 + np4;
      const float4* F4 = reinterpret_cast<const float4*>(a.M2F + (int64_t)s0 * fsz);
      for (int base = 0; base < ntot; base += 9 * BAND_NT) {
        float4 v[9];
#pragma unroll
        for (int u = 0; u < 9; ++u) {
          const int e = base + u * BAND_NT + tid;
          const int q = e - tb4;
          if (e < tb4) {
            v[u] = e < nbi4 ? Tsrc[e] : Wsrc[e - nbi4];
          } else if (q < nf4 || e >= ntot) {
            v[u] = F4[(q < nf4 && q >= 0) ? q : 0];
          } else {
            const int qq = q - nf4, i = qq / pp4, rem = qq - i * pp4, r = rem / nc4, n = rem - r * nc4, j = r >> 1;
            const BandSamplePts& sp = a.sp[(a.cofs + (s0 + i) / H) / a.C];
            v[u] = j < sp.n ? reinterpret_cast<const float4*>(a.tds + (2 * sp.p[j].kd + (r & 1)) * NCOL)[n]
                            : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int u = 0; u < 9; ++u) {
          const int e = base + u * BAND_NT + tid;
          const int q = e - tb4;
          if (e < tb4) {
            if (e < nbi4)
              reinterpret_cast<float4*>(Bimg)[e] = v[u];
            else
              reinterpret_cast<float4*>(twW)[e - nbi4] = v[u];
          } else if (q < nf4) {
            reinterpret_cast<float4*>(Fs)[q] = v[u];
          } else if (e < ntot) {
            reinterpret_cast<float4*>(Ps)[q - nf4] = v[u];
          }
        }
      }
      tb4 = 0;
      if (tid < nb * BAND_MAX_PTS) {
        const int i = tid / BAND_MAX_PTS, j = tid - i * BAND_MAX_PTS;
        const BandSamplePts& sp = a.sp[(a.cofs + (s0 + i) / H) / a.C];
        Pkw[tid] = j < sp.n ? (int)sp.p[j].kw : 0;
      }
    }
    __syncthreads();
    if (diag & 32) return;  // measurement: launch + first batch prologue only
    for (int un = c0 + ((wv - ((c0 - ub) & 3)) & 3); un < c1; un += 4) {  // (un - ub) % 4 == wave
      const int slab = un / ntw, tw_ = un - slab * ntw, slot = slab - s0;
      const int bcl = slab / H, h = slab - bcl * H, bc = a.bc0 + bcl;
      const float* F = Fs + slot * fsz + lane;  // fragment of (vt, ks): F[(vt KV + ks) 64]
      const float* Pr = Ps + slot * psz;
      const int w = 32 * tw_ + l31;
      const int wm = w % W;
      f32x16 vacc[VT];
#pragma unroll
      for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int j = 0; j < 16; ++j) vacc[vt][j] = 0.f;
      if (TB_INV_PRIO) __builtin_amdgcn_s_setprio(TB_INV_PRIO == 1 ? 2 : 0);
      int t = 0;
      const int kse = (diag & 4) ? 0 : KW + 1;
      int ks = 0;
      for (; ks + 4 <= kse; ks += 4) {  // the operands of 4 k-steps in flight before their MFMAs
        float fa[4][VT], bb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float2 c = twW[t];
          bb[q] = hl ? -c.y : c.x;
#pragma unroll
          for (int vt = 0; vt < VT; ++vt) fa[q][vt] = F[(vt * KV + ks + q) * 64];
          t += wm;
          t = t >= W ? t - W : t;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int vt = 0; vt < VT; ++vt)
            vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][vt], bb[q], vacc[vt], 0, 0, 0);
      }
      for (; ks < kse; ++ks) {
        const float2 c = twW[t];
        const float b = hl ? -c.y : c.x;
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
          vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(F[(vt * KV + ks) * 64], b, vacc[vt], 0, 0, 0);
        t += wm;
        t = t >= W ? t - W : t;
      }
      for (int j = 0; j < npm; ++j) {
        const int kw = Pkw[slot * BAND_MAX_PTS + j];
        const float2 c = twW[(kw * wm) % W];  // kw, wm < W <= 2^15
        const float b = hl ? -c.y : c.x;
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
          vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(F[(vt * KV + KW + 1 + j) * 64], b, vacc[vt], 0, 0, 0);
      }
      float* yb = a.y + (int64_t)bc * a.sbc + (int64_t)h * a.sh;
      const bool vec = ((a.sw & 3) == 0) && ((reinterpret_cast<uintptr_t>(yb) & 15) == 0);
      float lo = 3.402823466e38f, hi = -3.402823466e38f;
      // synthesis-table rows: < 2 NDk the band rows (Bimg), above them the slab's point rows and
      // four zero rows (the upper lane half reads up to 4 rows past nrv): B operands without branches
      const float* Tb = Bimg + l31;
      const float* Tp = Pr + l31 - 2 * NDk * NCOL;
      for (int nt = 0; nt < ntn; ++nt) {
        if (TB_INV_PRIO) __builtin_amdgcn_s_setprio(TB_INV_PRIO == 1 ? 2 : 0);
        f32x16 ye, yo;
#pragma unroll
        for (int j = 0; j < 16; ++j) ye[j] = yo[j] = 0.f;
        if (!(diag & 8))
#pragma unroll
          for (int vt = 0; vt < VT; ++vt) {
            // even sI: real rows (E); sI + 1: imaginary rows (O).  All 16 table operands are loaded
            // before the first MFMA (a step whose rows are past the used ones reads row 0 / 4 and
            // is skipped), so the LDS latency is paid once per tile, not once per k-step.
            float b0[8], b1[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int r = 32 * vt + acc_row(2 * i);
              const int re = (r < nrv ? r : 0) + 4 * hl;  // this lane's (real) row of the step
              const float* tr = (re < 2 * NDk ? Tb : Tp) + re * NCOL + nt * 32;
              b0[i] = tr[0];
              b1[i] = tr[NCOL];
            }
            if (32 * vt + acc_row(14) < nrv) {  // every step used (C3): one straight-line block
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                ye = __builtin_amdgcn_mfma_f32_32x32x2f32(b0[i], vacc[vt][2 * i], ye, 0, 0, 0);
                yo = __builtin_amdgcn_mfma_f32_32x32x2f32(b1[i], vacc[vt][2 * i + 1], yo, 0, 0, 0);
              }
            } else {
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                if (32 * vt + acc_row(2 * i) >= nrv) break;  // both halves' rows past the used ones are zero
                ye = __builtin_amdgcn_mfma_f32_32x32x2f32(b0[i], vacc[vt][2 * i], ye, 0, 0, 0);
                yo = __builtin_amdgcn_mfma_f32_32x32x2f32(b1[i], vacc[vt][2 * i + 1], yo, 0, 0, 0);
              }
            }
          }
        if (TB_INV_PRIO) __builtin_amdgcn_s_setprio(TB_INV_PRIO == 1 ? 0 : 2);
        if (diag & 16) continue;
        // y[w][d] = E - O (direct half), then y[w][D - d] = E + O (mirror half), each staged
        // [row][32] through LDS so that every store instruction writes whole 128-B row segments
        const int c4 = lane & 7;
        const int dbase = nt * 32 + 4 * c4, dmir = nt * 32 + 31 - 4 * c4;
        // the mirror of d = 0 is column D: the first U-Net pad column, written as 0 in the same vector
        const bool padlane = nt == 0 && c4 == 7 && ypad > 0;
        int nd = 0, nm = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          nd += dbase + q < Dh ? 1 : 0;
          const int d = dmir - q;
          nm += ((d >= 1 && 2 * d < D && d < Dh) || (padlane && d == 0)) ? 1 : 0;
        }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (half == 0)
                v[q] = ye[4 * g + q] - yo[4 * g + q];
              else
                v[3 - q] = ye[4 * g + q] + yo[4 * g + q];
            }
            const int col = half == 0 ? 8 * g + 4 * hl : 28 - 8 * g - 4 * hl;
            *reinterpret_cast<f32x4*>(stg + l31 * BAND_STG_P + col) = v;
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int r = (lane >> 3) + 8 * k;
            const int wr = 32 * tw_ + r;
            if (wr >= W) continue;
            f32x4 v = *reinterpret_cast<const f32x4*>(stg + r * BAND_STG_P + 4 * c4);
            float* yrr = yb + (int64_t)wr * a.sw;
            if (half == 0) {
              if (vec && nd == 4) {
                *reinterpret_cast<f32x4*>(yrr + dbase) = v;
                lo = fminf(lo, fminf(fminf(v[0], v[1]), fminf(v[2], v[3])));
                hi = fmaxf(hi, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
              } else if (nd > 0) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  if (q < nd) {
                    yrr[dbase + q] = v[q];
                    lo = fminf(lo, v[q]);
                    hi = fmaxf(hi, v[q]);
                  }
              }
            } else {
              if (padlane) v[3] = 0.f;  // column D
              if (vec && mal && nm == 4) {
                *reinterpret_cast<f32x4*>(yrr + D - dmir) = v;
                const float m3 = padlane ? v[2] : v[3];  // the pad zero is not an image value
                lo = fminf(lo, fminf(fminf(v[0], v[1]), fminf(v[2], m3)));
                hi = fmaxf(hi, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], m3)));
              } else if (nm > 0) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  const int d = dmir - q;  // v[q] is the value at column D - dmir + q = D - d
                  if (d >= 1 && 2 * d < D && d < Dh) {
                    yrr[D - d] = v[q];
                    lo = fminf(lo, v[q]);
                    hi = fmaxf(hi, v[q]);
                  } else if (padlane && d == 0) {
                    yrr[D] = 0.f;
                  }
                }
              }
              if (padlane) {  // the rest of the zero D-padding: columns D + 1 .. D + ypad - 1
                int p = 1;
                for (; p < ypad && ((D + p) & 3); ++p) yrr[D + p] = 0.f;
                if (vec)
                  for (; p + 4 <= ypad; p += 4) *reinterpret_cast<f32x4*>(yrr + D + p) = f32x4{0.f, 0.f, 0.f, 0.f};
                for (; p < ypad; ++p) yrr[D + p] = 0.f;
              }
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
      }
      if (a.mm) {  // per-unit partial (reduced per sample by k_band_minmax)
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane == 0) a.mmp[(int64_t)slab * ntw + tw_] = make_float2(lo, hi);
      }
    }
    c0 = c1;
  }
}

// ----------------------------------------------------------------------------- pass C' (split f16)
// The C2R synthesis in split precision on the f16 matrix cores (16x the f32 MFMA rate), unfolded:
//   Y^T(w, d) = sum_v V^T(w, v) T(v, d),   T(2 kd, d) = cos(2 pi kd d / D), T(2 kd + 1, d) = -sin(..)
// for every output column d < D + pad (T = 0 past D: the U-Net's zero padding comes out of the
// MFMA).  V^T is the V-product accumulator tile used as the A operand as it stands (its rows are
// the k index); T is the launch's fragment image (band_tab16, built by pass B2''s extra blocks) in LDS.  Split precision:
// V = Vh + Vl (scaled by a power of two per unit so that max |V| < 2^15), T = Th + Tl (scaled by
// 2^8), Y = (Vh Th + Vh Tl + Vl Th) / scale -- 22 bits per operand, the dropped Vl Tl term
// 2^-22 relative, so Y matches the f32 synthesis to a few 1e-7 of max |y|.  The accumulator has
// the image row w in its registers and the column d on the lane, so each register is stored
// straight to HBM as two whole 128-B row segments: no LDS staging, no mirror stores.
constexpr float BAND_T16_SCALE = 256.f;

// One thread per (column tile, 16-row chunk, lane): the lane's 8 B-fragment entries of T, k-permuted
// to match the accumulator-as-A-operand order of V^T (element j of lane half h is V row
// 16 c + 8 (j >> 2) + 4 h + (j & 3)); rows 2 kd + (re, im), the band columns first, then every
// sample's out-of-box points in launch order.
__device__ void band_tab16(const BandMidArgs& a, int t) {
  const int nch = band_nch(a.g), ntd = a.g.NTD, NCOL = a.g.NCOL, NDk = a.g.NDk, D = a.pl.D, Dh = D / 2 + 1;
  if (t >= ntd * nch * 64) return;
  const int lane = t & 63, cc = t >> 6, c = cc % nch, nt = cc / nch;
  const int d = 32 * nt + (lane & 31), hl = lane >> 5;
  // column d of the unfolded table from the folded one: d > D/2 mirrors to D - d (sin changes sign)
  const bool in = d < D, mir = d >= Dh;
  const int dd = mir ? D - d : d;
  h16x8 fh, fl;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int v = 16 * c + 8 * (j >> 2) + 4 * hl + (j & 3);
    const int pr = v >> 1, im = v & 1;
    const int kd = pr < NDk ? pr : (pr - NDk < a.g.PT ? (int)a.pkd[pr - NDk] : -1);
    float tv = 0.f;
    if (kd >= 0 && in) {
      tv = a.tds[(2 * kd + im) * NCOL + dd];
      if (im && !mir) tv = -tv;  // -sin(2 pi kd d / D) = +sin(2 pi kd (D - d) / D)
    }
    _Float16 h, l;
    split_f16(tv * BAND_T16_SCALE, h, l);
    fh[j] = h;
    fl[j] = l;
  }
  h16x8* T = reinterpret_cast<h16x8*>(a.T16);
  T[(cc * 2) * 64 + lane] = fh;
  T[(cc * 2 + 1) * 64 + lane] = fl;
}

#ifndef TB_INV16_WPE
#define TB_INV16_WPE 4  // waves per SIMD the VT = 1 split-f16 kernel is compiled for (register budget)
#endif
#ifndef TB_INV16_NW
#define TB_INV16_NW 16  // waves per split-f16 pass-C' workgroup: 16 = one workgroup per CU (C3 80 -> 72 us vs 4)
#endif
#ifndef TB_INV16_TR
#define TB_INV16_TR 1   // 1: tile rows = image columns where row strides allow (see k_band_inv16); 0: never; 2: always
#endif
#ifndef TB_INV16_NTS
#define TB_INV16_NTS 0  // 1: C''s whole-line stores non-temporal
#endif
#ifndef TB_INV16_SWZ
#define TB_INV16_SWZ 1  // 1: C' tiles regrouped across lanes so each 16-B store instruction writes 8 whole rows
#endif
// A 32 x 32 output tile in the TR layout -- lane (w = lane & 31, half = lane >> 5), register group g:
// row w, columns 8 g + 4 half + 0..3 -- leaves each store instruction 32 rows x 32 B (128 partial
// lines).  Two exchanges regroup it so that o[k] holds rows 8 k + (lane & 7), columns
// 16 ((lane >> 3) & 1) + {0, 8, 4, 12}[lane >> 4] + 0..3: 8 whole 128-B rows per instruction.
//   permlane16_swap(v[g], v[g+1]) (g = 0, 2): the odd 16-lane rows of v[g] trade with the even rows
//   of v[g+1] -> v[g]: rows 0..15, columns 8 g + 0..15 (4 lanes a row), v[g+1]: rows 16..31;
//   row_ror:8 inside each 16-lane row, written to one half of the banks, pairs rows r and r + 8.
__device__ __forceinline__ void tile_rows8(const f32x4 (&v)[4], f32x4 (&o)[4]) {
  f32x4 t[4];
#pragma unroll
  for (int g = 0; g < 4; g += 2)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[g][q]), __float_as_uint(v[g + 1][q]), false,
                                                      false);
      t[g][q] = __uint_as_float(r[0]);      // rows 0..15, columns 8 g + ..
      t[g + 1][q] = __uint_as_float(r[1]);  // rows 16..31
    }
#pragma unroll
  for (int h = 0; h < 2; ++h)  // h = 0: rows 0..15 (t[0] columns 0..15, t[2] 16..31), h = 1: rows 16..31
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned lo = __float_as_uint(t[h][q]), hi = __float_as_uint(t[2 + h][q]);
      o[2 * h][q] = __uint_as_float(__builtin_amdgcn_update_dpp(lo, hi, 0x128, 0xF, 0xC, false));
      o[2 * h + 1][q] = __uint_as_float(__builtin_amdgcn_update_dpp(hi, lo, 0x128, 0xF, 0x3, false));
    }
}

template <int VT, int NW, bool TR>  // 32-row tiles of V; waves per workgroup; tile rows = image columns
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(VT == 1 ? TB_INV16_WPE : 3, 8))) void k_band_inv16(BandInvArgs) {
  // Same unit structure as k_band_inv: (slab, 32-row tile) units dealt to a persistent grid, each
  // workgroup's slabs in batches whose V-product fragments are loaded to LDS first (the unit loop
  // then issues no vector-memory loads), per-unit min/max partials.
  const BandInvArgs& a = kargs<BandInvArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63, hl = lane >> 5, l31 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int KW = a.g.KW;
  const int npm = a.g.KS - a.g.NDk;    // point k-steps of the V product (max points per sample)
  const int KV = KW + 1 + npm;
  const int nch = band_nch(a.g);       // 16-row chunks of V in use
  const int ntd = a.g.NTD;             // 32-column tiles of the output row (D + pad)
  const int fsz = VT * KV * 64;
  constexpr int NT = 64 * NW;
  const int SLOTS = a.slots;  // slabs per fragment batch (launch_inv16_t: the workgroup's whole range where LDS allows)
  const BandInv16Carve cv = band_inv16_carve(a.g, W, SLOTS);
  const h16x8* Tab = reinterpret_cast<const h16x8*>(smem + cv.tab);  // [nt][c][hi/lo][64]
  float2* twW = reinterpret_cast<float2*>(smem + cv.tww);
  float* Fs = reinterpret_cast<float*>(smem + cv.frag);
  int* Pkw = reinterpret_cast<int*>(smem + cv.pkw);
  const int ntab4 = band_t16_bytes(a.g) / 16;
  const bool twv = !(W & 1) && (reinterpret_cast<uintptr_t>(a.pl.tw[1]) & 15) == 0;
  const int ntw4 = twv ? W / 2 : 0;
  if (!twv)
    for (int i = tid; i < W; i += NT) twW[i] = reinterpret_cast<const float2*>(a.pl.tw[1])[i];
  const float4* Tsrc = reinterpret_cast<const float4*>(a.T16);
  const float4* Wsrc = reinterpret_cast<const float4*>(a.pl.tw[1]);
  int tb4 = ntab4 + ntw4;
  const int ntw = (W + 31) / 32;
  const int nslab = H * a.nbc;
  const int ncolo = D + a.ypad;        // stored columns of a row
  if (a.diag & 128) tb4 = 0;           // measurement: no table loads (results invalid)
  const int diag = a.diag;             // measurement only (TEXBIAS_BAND_DIAG >> 8): skipped stages
  constexpr bool tr = TR;
  if (diag & 64) return;
  const int nunit = nslab * ntw;
  const int per = (nunit + (int)gridDim.x - 1) / (int)gridDim.x;
  const int ub = (int)blockIdx.x * per, ue = ub + per < nunit ? ub + per : nunit;
  __shared__ uint32_t kmm[2 * TB_MAX_BATCH];  // this workgroup's per-sample (min, max) keys
  if (tid < 2 * TB_MAX_BATCH) kmm[tid] = (tid & 1) ? 0u : 0xffffffffu;
  __syncthreads();
  for (int c0 = ub; c0 < ue;) {
    const int s0 = c0 / ntw;
    const int slast = (ue - 1) / ntw;
    const int s1 = slast < s0 + SLOTS - 1 ? slast : s0 + SLOTS - 1;
    const int c1 = (s1 + 1) * ntw < ue ? (s1 + 1) * ntw : ue;
    const int nb = s1 - s0 + 1;
    __syncthreads();
    {  // [tables,] the batch's V-product fragments: rounds of loads in flight
      const int nf4 = (a.diag & 256) ? 0 : nb * fsz / 4;
      const int ntot = tb4 + nf4;
      const float4* F4 = reinterpret_cast<const float4*>(a.M2F + (int64_t)s0 * fsz);
      // source and LDS destination chosen by selects, every load unconditional (a clamped index):
      // branches around the loads made the compiler keep v[] in scratch and wait on each load
      for (int base = 0; base < ntot; base += 9 * NT) {
        float4 v[9];
#pragma unroll
        for (int u = 0; u < 9; ++u) {
          const int e = base + u * NT + tid;
          const int q = e - tb4;
          const float4* src = e < tb4 ? (e < ntab4 ? Tsrc + e : Wsrc + (e - ntab4)) : F4 + (q < nf4 ? q : 0);
          v[u] = *src;
        }
#pragma unroll
        for (int u = 0; u < 9; ++u) {
          const int e = base + u * NT + tid;
          const int q = e - tb4;
          const int dst = e < tb4 ? (e < ntab4 ? cv.tab + 16 * e : cv.tww + 16 * (e - ntab4)) : cv.frag + 16 * q;
          if (e < tb4 || q < nf4) *reinterpret_cast<float4*>(smem + dst) = v[u];
        }
      }
      tb4 = 0;
      if (tid < nb * BAND_MAX_PTS) {
        const int i = tid / BAND_MAX_PTS, j = tid - i * BAND_MAX_PTS;
        const BandSamplePts& sp = a.sp[(a.cofs + (s0 + i) / H) / a.C];
        Pkw[tid] = j < sp.n ? (int)sp.p[j].kw : 0;
      }
    }
    __syncthreads();
    if (diag & 32) return;
    for (int un = c0 + ((wv - ((c0 - ub) % NW) + NW) % NW); un < c1; un += NW) {  // (un - ub) % NW == wave
      const int slab = un / ntw, tw_ = un - slab * ntw, slot = slab - s0;
      const int bcl = slab / H, h = slab - bcl * H, bc = a.bc0 + bcl;
      const float* F = Fs + slot * fsz + lane;
      const int w = 32 * tw_ + l31;
      const int wm = w % W;
      f32x16 vacc[VT];
#pragma unroll
      for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int j = 0; j < 16; ++j) vacc[vt][j] = 0.f;
      int t = 0;
      int ks = 0;
      const int kse = (diag & 4) ? 0 : KW + 1;
      for (; ks + 4 <= kse; ks += 4) {
        float fa[4][VT], bb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float2 c = twW[t];
          bb[q] = hl ? -c.y : c.x;
#pragma unroll
          for (int vt = 0; vt < VT; ++vt) fa[q][vt] = F[(vt * KV + ks + q) * 64];
          t += wm;
          t = t >= W ? t - W : t;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int vt = 0; vt < VT; ++vt)
            vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][vt], bb[q], vacc[vt], 0, 0, 0);
      }
      for (; ks < kse; ++ks) {
        const float2 c = twW[t];
        const float b = hl ? -c.y : c.x;
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
          vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(F[(vt * KV + ks) * 64], b, vacc[vt], 0, 0, 0);
        t += wm;
        t = t >= W ? t - W : t;
      }
      for (int j = 0; j < (kse ? npm : 0); ++j) {
        const int kw = Pkw[slot * BAND_MAX_PTS + j];
        const float2 c = twW[(kw * wm) % W];
        const float b = hl ? -c.y : c.x;
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
          vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(F[(vt * KV + KW + 1 + j) * 64], b, vacc[vt], 0, 0, 0);
      }
      // V^T as split-f16 A operands: chunk c = 2 vt + q is registers 8 q .. 8 q + 7 of vacc[vt]
      float m = 0.f;
#pragma unroll
      for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int j = 0; j < 16; ++j) m = fmaxf(m, fabsf(vacc[vt][j]));
      m = wave_max(m);
      int ex;
      (void)frexpf(m, &ex);  // m < 2^ex
      const float sv = ldexpf(1.f, 15 - ex), inv = ldexpf(1.f, ex - 15) * (1.f / BAND_T16_SCALE);
      h16x8 ah[2 * VT], al[2 * VT];
#pragma unroll
      for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            _Float16 hh, ll;
            split_f16(vacc[vt][8 * q + j] * sv, hh, ll);
            ah[2 * vt + q][j] = hh;
            al[2 * vt + q][j] = ll;
          }
      float* yb = a.y + (int64_t)bc * a.sbc + (int64_t)h * a.sh;
      float lo = 3.402823466e38f, hi = -3.402823466e38f;
      const int wb = 32 * tw_ + 4 * hl;  // image row of accumulator register r: wb + acc_row(r)
      // regrouped tile (tile_rows8): lane's row 32 tw + 8 k + (lane & 7), column offset cs0 + 32 nt
      const int r8 = 32 * tw_ + (lane & 7);
      const int cs0 = 16 * ((lane >> 3) & 1) + ((0xC480 >> (4 * (lane >> 4))) & 15);
      float* ys = yb + (int64_t)(r8 < W ? r8 : 0) * a.sw + cs0;
      const int64_t s8 = 8 * a.sw;
      for (int nt = 0; nt < ntd; ++nt) {
        f32x16 acc;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
        for (int c = 0; c < 2 * VT; ++c) {
          if (c >= nch || (diag & 8)) break;
          const h16x8* tp = Tab + ((nt * nch + c) * 2) * 64 + lane;
          const h16x8 th = tp[0], tl = tp[64];
          if (tr) {  // Y(d, w) = T(d, v) . V(v, w): the table as the A operand, the V tile as B
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, al[c], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, ah[c], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ah[c], acc, 0, 0, 0);
          } else {   // Y^T(w, d) = V^T(w, v) . T(v, d)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[c], th, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], tl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], th, acc, 0, 0, 0);
          }
        }
        const int col = 32 * nt + l31;
        if (diag & 16) {  // no stores: keep the results live
          float z = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) z += acc[r];
          lo = fminf(lo, z);
          continue;
        }
        if (tr) {  // lane (w, half): columns 32 nt + 8 g + 4 half + 0..3 in registers 4 g .. 4 g + 3: 16-B stores
          const int wr = 32 * tw_ + l31;
          const bool vec = ((a.sw & 3) == 0) && ((reinterpret_cast<uintptr_t>(yb) & 15) == 0);
          f32x4 v[4];
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[g][q] = acc[4 * g + q] * inv;  // exactly 0 past D (T = 0 there)
          if (TB_INV16_SWZ && vec && 32 * nt + 32 <= ncolo) {  // wave-uniform: whole 128-B lines per store
            f32x4 o[4];
            tile_rows8(v, o);
            const bool img = 32 * nt + 32 <= D;  // wave-uniform: every column an image column
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if (r8 + 8 * k < W) {
                f32x4* dst = reinterpret_cast<f32x4*>(ys + k * s8 + 32 * nt);
                if (TB_INV16_NTS) __builtin_nontemporal_store(o[k], dst);
                else *dst = o[k];
                if (img) {
#pragma unroll
                  for (int q = 0; q < 4; ++q) {
                    lo = fminf(lo, o[k][q]);
                    hi = fmaxf(hi, o[k][q]);
                  }
                } else {
#pragma unroll
                  for (int q = 0; q < 4; ++q)
                    if (32 * nt + cs0 + q < D) {
                      lo = fminf(lo, o[k][q]);
                      hi = fmaxf(hi, o[k][q]);
                    }
                }
              }
            }
            continue;
          }
          if (wr < W) {
            float* yr = yb + (int64_t)wr * a.sw;
            if (vec && 32 * nt + 32 <= ncolo) {  // wave-uniform: the whole tile lies inside the row
#pragma unroll
              for (int g = 0; g < 4; ++g) *reinterpret_cast<f32x4*>(yr + 32 * nt + 8 * g + 4 * hl) = v[g];
            } else {
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const int d0 = 32 * nt + 8 * g + 4 * hl;
                if (vec && d0 + 4 <= ncolo) {
                  *reinterpret_cast<f32x4*>(yr + d0) = v[g];
                } else {
#pragma unroll
                  for (int q = 0; q < 4; ++q)
                    if (d0 + q < ncolo) yr[d0 + q] = v[g][q];
                }
              }
            }
            if (32 * nt + 32 <= D) {  // wave-uniform: every column an image column -- min3/max3 chains
#pragma unroll
              for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  lo = fminf(lo, v[g][q]);
                  hi = fmaxf(hi, v[g][q]);
                }
            } else {
#pragma unroll
              for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  if (32 * nt + 8 * g + 4 * hl + q < D) {
                    lo = fminf(lo, v[g][q]);
                    hi = fmaxf(hi, v[g][q]);
                  }
            }
          }
          continue;
        }
        if (col < ncolo) {
          float* yc = yb + col;
          const bool img = col < D;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int wr = wb + acc_row(r);
            if (wr < W) {
              const float v = acc[r] * inv;  // exactly 0 in the pad columns (T = 0 there)
              yc[(int64_t)wr * a.sw] = v;
              if (img) {
                lo = fminf(lo, v);
                hi = fmaxf(hi, v);
              }
            }
          }
        }
      }
      if (a.mm) {  // the unit's (min, max) into the workgroup's per-sample keys (LDS atomics)
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane == 0) {
          const int sl = bcl / a.C;  // sample of the launch
          atomicMin(&kmm[2 * sl], f2key(lo));
          atomicMax(&kmm[2 * sl + 1], f2key(hi));
        }
      }
    }
    c0 = c1;
  }
  // one device-scope atomic pair per (workgroup, sample) onto the keys pass B' initialised: no partials,
  // no last-arriver reduction in the kernel's tail (round 5's hand-off cost C' ~3 us at its end)
  __syncthreads();
  if (a.mm && (int)threadIdx.x < a.nbc / a.C && kmm[2 * threadIdx.x] != 0xffffffffu) {
    const int sk = a.bc0 / a.C + (int)threadIdx.x;
    atomicMin(&a.mm[2 * sk], kmm[2 * threadIdx.x]);
    atomicMax(&a.mm[2 * sk + 1], kmm[2 * threadIdx.x + 1]);
  }
}

// per-sample keys of the slab partials: one workgroup per sample
__global__ __launch_bounds__(256) void k_band_minmax(const float2* __restrict__ mmp, uint32_t* __restrict__ mm, int bc0,
                                                     int C, int H, int W) {
  __shared__ float red[2 * 256 / 64];
  const int b = (int)blockIdx.x;
  const int ntw = (W + 31) / 32;
  const int64_t n = (int64_t)C * H * ntw;  // one partial per (slab, 32-row tile)
  const float2* p = mmp + (int64_t)b * C * H * ntw;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  int64_t i0 = 0;
  if (((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {  // two partials per 16-B load, 4 loads in flight
    const float4* p4 = reinterpret_cast<const float4*>(p);
    const int64_t n4 = n / 2;
    for (int64_t j = threadIdx.x; j < n4; j += 4 * 256) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = j + u * 256 < n4 ? p4[j + u * 256] : make_float4(lo, hi, lo, hi);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        lo = fminf(lo, fminf(v[u].x, v[u].z));
        hi = fmaxf(hi, fmaxf(v[u].y, v[u].w));
      }
    }
    i0 = 2 * n4;
  }
  for (int64_t i = i0 + threadIdx.x; i < n; i += 256) {
    const float2 v = p[i];
    lo = fminf(lo, v.x);
    hi = fmaxf(hi, v.y);
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[wid] = lo;
    red[4 + wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      lo = fminf(lo, red[w]);
      hi = fmaxf(hi, red[4 + w]);
    }
    const int sb = bc0 / C + b;
    mm[2 * sb] = f2key(lo);
    mm[2 * sb + 1] = f2key(hi);
  }
}

// ----------------------------------------------------------------------------- identity
__global__ __launch_bounds__(256) void k_copy_pad(CopyArgs a) {
  __shared__ float red[2 * 256 / 64];
  const int tid = (int)threadIdx.x;
  const int units = a.H * a.nbc;
  const int len = a.D + a.ypad;
  const FastDiv fl = FastDiv::make(len);
  const bool same = a.x == a.y && a.xsbc == a.ysbc && a.xsh == a.ysh && a.xsw == a.ysw;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int u = (int)blockIdx.x; u < units; u += (int)gridDim.x) {
    const int bcl = u / a.H, h = u - bcl * a.H, bc = a.bc0 + bcl;
    const float* xb = a.x + (int64_t)bc * a.xsbc + (int64_t)h * a.xsh;
    float* yb = a.y + (int64_t)bc * a.ysbc + (int64_t)h * a.ysh;
    for (int e = tid; e < a.W * len; e += 256) {
      const int w = fl.div(e), d = e - w * len;
      if (d < a.D) {
        const float v = xb[(int64_t)w * a.xsw + d];
        if (!same) yb[(int64_t)w * a.ysw + d] = v;
        lo = fminf(lo, v);
        hi = fmaxf(hi, v);
      } else {
        yb[(int64_t)w * a.ysw + d] = 0.f;
      }
    }
    const int un = u + (int)gridDim.x;
    const int b = bc / a.C;
    if (a.mm && (un >= units || (a.bc0 + un / a.H) / a.C != b)) {
      block_minmax_atomic<256>(lo, hi, red, a.mm + 2 * b);
      lo = 3.402823466e38f;
      hi = -3.402823466e38f;
    }
  }
}

// Persistent grid: the workgroups that are resident at once (LDS and register occupancy, at most
// 4 per CU), never more than there are units -- no second, partial round of workgroups.
// Occupancy per (kernel, LDS bytes), computed once and cached under a lock (host threads may drive
// one device each; the instantiations of one template share a function type, so the kernel's
// address is part of the key).
template <class K>
int band_occupancy(K kern, size_t lds, int nt, int cap) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  const auto key = std::make_pair(reinterpret_cast<const void*>(kern), lds);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, nt, lds) != hipSuccess || occ < 1)
    occ = (int)(163840 / (lds ? lds : 1));
  occ = occ < 1 ? 1 : (occ > cap ? cap : occ);
  cache[key] = occ;
  return occ;
}

template <class K>
int band_grid(K kern, int units, size_t lds, int ncu, int cap = 4) {
  const int per_cu = band_occupancy(kern, lds, BAND_NT, cap);
  const int g = ncu * per_cu;
  return units < g ? units : g;
}

template <int NT2, int KWT, int DC, bool F16 = false>
hipError_t launch_fwd_t(BandFwdArgs& a, size_t lds, int ncu, hipStream_t st) {
  auto kern = k_band_fwd<NT2, KWT, DC, F16>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  // waves: as many as are resident at once (LDS / register occupancy), but at most T / ceil(nst / 2)
  // so that a slab spans at most BAND_FWD_SEGS waves, and (T + 1) G < 2^32 for the 32-bit split
  const int last_occ = band_occupancy(kern, lds, BAND_NT, 8);
  const uint32_t nst = (uint32_t)((a.pl.W + BAND_FWD_ROWS - 1) / BAND_FWD_ROWS);
  const uint64_t T = (uint64_t)a.pl.H * (uint64_t)a.nbc * nst;
  uint64_t G = (uint64_t)ncu * (uint64_t)last_occ * 4;
  const uint64_t gmax = T / ((nst + 1) / 2);
  G = G < gmax ? G : gmax;
  while (G > 1 && (T + 1) * G >= (1ull << 32)) G >>= 1;
  if (G < 1) G = 1;
  if (T >= (1ull << 31)) return hipErrorInvalidValue;
  a.split = FwdSplit{(uint32_t)T, (uint32_t)G, nst};
  hipLaunchKernelGGL(kern, dim3((unsigned)((G + 3) / 4)), dim3(BAND_NT), lds, st, a);
  return hipGetLastError();
}

template <int VT, int NW>
hipError_t launch_inv16_t(BandInvArgs& a, int ncu, hipStream_t st) {
  // slab slots: a 16-wave workgroup (one per CU) holds every slab of its unit range when LDS allows,
  // so its units run after ONE fragment batch (C2: 32 slabs per workgroup, 3 batches of 12 before)
  int slots = band_slots16(NW);
  if (NW == 16) {
    const int ntw = (a.pl.W + 31) / 32, nslab = a.pl.H * a.nbc;
    const int grid = nslab < ncu ? nslab : ncu;
    const int per = (nslab * ntw + grid - 1) / grid;
    const int want = (per + ntw - 1) / ntw + 1;  // a range may start and end inside a slab
    while (slots < want && band_inv16_carve(a.g, a.pl.W, slots + 1).total <= 160000) ++slots;
  }
  a.slots = slots;
  const size_t lds = band_inv16_carve(a.g, a.pl.W, slots).total;
  // output orientation: tile rows = image columns.  With 16-B aligned rows the tile is regrouped
  // into whole-line stores (tile_rows8), which beat the image-row orientation at every row stride
  // (C2, 512-B rows: 77 -> 69 us).  Without them the 32 x 32-B pieces of a store pile onto one
  // memory channel when rows are 512-B strided: those keep image rows.
  const bool swz_ok = TB_INV16_SWZ && (a.sw & 3) == 0 && (a.sbc & 3) == 0 && (a.sh & 3) == 0 &&
                      (reinterpret_cast<uintptr_t>(a.y) & 15) == 0;
  auto kern = (TB_INV16_TR == 2 || (TB_INV16_TR && (swz_ok || ((a.sw * 4) % 512) != 0))) ? k_band_inv16<VT, NW, true> : k_band_inv16<VT, NW, false>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int per_cu = band_occupancy(kern, lds, 64 * NW, 8);
  const int units = a.pl.H * a.nbc, g = ncu * per_cu;
  hipLaunchKernelGGL(kern, dim3(units < g ? units : g), dim3(64 * NW), lds, st, a);
  return hipGetLastError();
}

template <int VT>
hipError_t launch_inv_t(const BandInvArgs& a, int ncu, hipStream_t st) {
  const size_t lds = band_inv_carve(a.g, a.pl.W, a.pl.D).total;
  auto kern = k_band_inv<VT>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int units = a.pl.H * a.nbc;  // slabs, taken in batches of BAND_SLOTS per workgroup
  hipLaunchKernelGGL(kern, dim3(band_grid(kern, units, lds, ncu)), dim3(BAND_NT), lds, st, a);
  return hipGetLastError();
}

}  // namespace

bool band_fwd_use_ct(int D, int NT2) {
  return band_fwd_ct(D, NT2);
}

hipError_t launch_band_fwd(BandFwdArgs& a, int ncu, hipStream_t st) {
  const bool n1 = a.g.NDk <= 16, k1 = a.g.KW < 16;
  const bool ct = band_fwd_use_ct(a.pl.D, n1 ? 1 : 2);
  const size_t lds = band_lds_fwd(a.g, a.pl.W, a.pl.D, ct);
  if (ct) {
    // split-f16 D product for D = 155 (C3: 63.2 -> 61.6 us with flushed caches, level in the train-step
    // bench); D = 128 (C2) keeps the f32 product (its 8 KB strips: 57.9 vs 59.6 us in the C2 bench)
    const bool f16 = a.tbt16 && a.vec && a.pl.D == 155;
    const size_t lds16 = lds + (size_t)band_fwd16_ks(a.pl.D) * 4 * 64 * 16 - (((size_t)a.pl.W * 8 + 15) & ~(size_t)15);
    if (f16) return k1 ? launch_fwd_t<1, 1, 155, true>(a, lds16, ncu, st) : launch_fwd_t<1, 2, 155, true>(a, lds16, ncu, st);
    if (a.pl.D == 155) {
      return k1 ? launch_fwd_t<1, 1, 155>(a, lds, ncu, st) : launch_fwd_t<1, 2, 155>(a, lds, ncu, st);
    }
    return k1 ? launch_fwd_t<1, 1, 128>(a, lds, ncu, st) : launch_fwd_t<1, 2, 128>(a, lds, ncu, st);
  }
  if (n1) return k1 ? launch_fwd_t<1, 1, 0>(a, lds, ncu, st) : launch_fwd_t<1, 2, 0>(a, lds, ncu, st);
  return k1 ? launch_fwd_t<2, 1, 0>(a, lds, ncu, st) : launch_fwd_t<2, 2, 0>(a, lds, ncu, st);
}

template <int MT>
hipError_t launch_hcol_t(const BandMidArgs& a, hipStream_t st) {
  const size_t lds = band_hc_lds(a.pl.H, a.g.KH);
  auto kern = k_band_hcol<MT>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((a.g.ncol + BAND_HC_CB - 1) / BAND_HC_CB, a.nbc), dim3(64 * BAND_HC_NW), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_band_mid(const BandMidArgs& a, hipStream_t st) {
  hipError_t e = a.g.KH + 1 <= 16 ? launch_hcol_t<1>(a, st) : launch_hcol_t<2>(a, st);
  if (e != hipSuccess) return e;
  const int ntab = a.g.cat ? (a.g.NTD * band_nch(a.g) * 64 + BAND_NT - 1) / BAND_NT : 0;
  hipLaunchKernelGGL(k_band_zh, dim3((a.pl.H * a.nbc + 3) / 4 + ntab), dim3(BAND_NT), 0, st, a);
  return hipGetLastError();
}



hipError_t launch_band_inv(BandInvArgs& a, int ncu, hipStream_t st) {
  if (a.g.cat) {
    if (TB_INV16_NW == 16 && band_inv16_carve(a.g, a.pl.W, band_slots16(16)).total <= 160000)
      return band_vt(a.g) == 1 ? launch_inv16_t<1, 16>(a, ncu, st) : launch_inv16_t<2, 16>(a, ncu, st);
    return band_vt(a.g) == 1 ? launch_inv16_t<1, 4>(a, ncu, st) : launch_inv16_t<2, 4>(a, ncu, st);
  }
  return band_vt(a.g) == 1 ? launch_inv_t<1>(a, ncu, st) : launch_inv_t<2>(a, ncu, st);
}

hipError_t launch_band_minmax(const float2* mmp, uint32_t* mm, int bc0, int C, int nbc, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(k_band_minmax, dim3(nbc / C), dim3(256), 0, st, mmp, mm, bc0, C, H, W);
  return hipGetLastError();
}

hipError_t launch_copy_pad(const CopyArgs& a, hipStream_t st) {
  const int units = a.H * a.nbc;
  const int g = units < 2048 ? units : 2048;
  hipLaunchKernelGGL(k_copy_pad, dim3(g), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace tb
