// kern_band.hip -- the band-limited k-space passes A' / B' / C' (band.h) and the identity copy.
//
// Reference restated (file:line under /root/reference):
//   Fourier.shift_fourier / inv_shift_fourier     source_code/filters_and_operators.py:594-632
//   RandFourierDiskMaskd (low-pass disk)           source_code/filters_and_operators.py:236-279
//   RandPlaneWaves_ellipsoid / KSpaceSpikeNoise    :370-414 / :906-983 (point updates)
//   WrapArtifact, GibbsNoise, GibbsNoiseLayer      :503-515, :678-705, stylization_layers.py:91-116
// The op program is applied by apply_ops (fft_core.h), shared with the full-spectrum pass B.
#include <hip/hip_runtime.h>

#include "band.h"

namespace tb {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float2 ld2(const cf* p) {
  const cf v = *p;
  return make_float2(v.x, v.y);
}

// ----------------------------------------------------------------------------- pass A'
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BAND_PF = 10;  // 16-B (or 4-B) prefetch registers per lane: 64 rows x D <= 2560 floats

// One 64-row chunk of a slab: where its rows start and how they are laid out in memory.
struct ChunkSrc {
  const float* src;  // first element of the chunk's first row
  int total;         // rows * D
  int off;           // contiguous rows: src - (16-B aligned start), in floats
  int nq;            // contiguous rows: 16-B vectors covering the chunk
};
__device__ __forceinline__ ChunkSrc chunk_src(const float* xb, int64_t sw, int w0, int nr, int D) {
  ChunkSrc c;
  c.src = xb + (int64_t)w0 * sw;
  c.total = nr * D;
  c.off = (int)((reinterpret_cast<uintptr_t>(c.src) >> 2) & 3);
  c.nq = (c.total + c.off + 3) >> 2;
  return c;
}
// Issue the chunk's global loads into registers (no LDS traffic): every lane keeps up to
// BAND_PF independent 16-B loads in flight while the current chunk is computed (contiguous rows).
__device__ __forceinline__ void chunk_load(f32x4 (&v)[BAND_PF], const ChunkSrc& c, int tid) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(c.src - c.off);
#pragma unroll
  for (int u = 0; u < BAND_PF; ++u) {
    const int q = tid + u * BAND_NT;
    if (q < c.nq) v[u] = __builtin_nontemporal_load(s4 + q);
  }
}
// Odd D (LDS pitch = D): the chunk is one contiguous run in LDS too, laid out so that element e
// sits at X[off + e] -- every 16-B global vector lands 16-B aligned in LDS (one ds_write_b128,
// no per-element index math); the chunk's base pointer is then X + off.  Even D (pitch D + 1 for
// conflict-free row reads) inserts one pad float per row.
__device__ __forceinline__ const float* chunk_store(float* X, const f32x4 (&v)[BAND_PF], const ChunkSrc& c, int D,
                                                    const FastDiv& fd, int tid) {
  if (D & 1) {
#pragma unroll
    for (int u = 0; u < BAND_PF; ++u) {
      const int q = tid + u * BAND_NT;
      if (q < c.nq) *reinterpret_cast<f32x4*>(X + 4 * q) = v[u];
    }
    return X + c.off;
  }
#pragma unroll
  for (int u = 0; u < BAND_PF; ++u) {
    const int e0 = 4 * (tid + u * BAND_NT) - c.off;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = e0 + k;
      if (e >= 0 && e < c.total) X[e + fd.div(e)] = v[u][k];
    }
  }
  return X;
}
// strided rows (e.g. the padded U-Net buffer filtered in place): plain copy, no prefetch
__device__ __forceinline__ void chunk_copy_strided(float* xs, int P, const ChunkSrc& c, int64_t sw, int D,
                                                   const FastDiv& fd, int tid) {
  for (int e0 = tid; e0 < c.total; e0 += 8 * BAND_NT) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = e0 + k * BAND_NT;
      if (e < c.total) {
        const int r = fd.div(e);
        v[k] = c.src[(int64_t)r * sw + (e - r * D)];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = e0 + k * BAND_NT;
      if (e < c.total) {
        const int r = fd.div(e);
        xs[r * P + (e - r * D)] = v[k];
      }
    }
  }
}

// NT2: 16-wide kd tiles (NDk <= 16 NT2); NI: stage-W items per thread ((KW+1) NDk <= 256 NI)
template <int NT2, int NI>
__global__ __launch_bounds__(BAND_NT) void k_band_fwd(BandFwdArgs) {
  const BandFwdArgs& a = kargs<BandFwdArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, ncol = a.g.ncol;
  const int P = (D & 1) ? D : D + 1;
  const int Ld = D / 2 + 1;                 // folded d in [0, D/2]
  const int KSd = (Ld + 3) / 4;             // 16x16x4 k-steps
  float* X = reinterpret_cast<float*>(smem);                                    // [64][P] (+8 slack)
  float2* Rb = reinterpret_cast<float2*>(X + BAND_ROWS_A * P + 8);              // [kd][65]
  float2* twW = Rb + NDk * (BAND_ROWS_A + 1);                                   // (cos, -sin)(2 pi t / W)
  float* Bt = reinterpret_cast<float*>(twW + W);                                // [NT2][KSd][2][64]
  for (int t = tid; t < W; t += BAND_NT) twW[t] = ld2(a.pl.tw[1] + t);
  // B fragments of the folded D product: lane l of k-step ks holds d = 4 ks + l/16, kd = 16 nt + l%16
  for (int e = tid; e < NT2 * KSd * 128; e += BAND_NT) {
    const int ln = e & 63, part = (e >> 6) & 1, ks = (e >> 7) % KSd, nt = (e >> 7) / KSd;
    const int d = 4 * ks + (ln >> 4), kd = 16 * nt + (ln & 15);
    float v = 0.f;
    if (d < Ld && kd < NDk) {
      const cf tw = a.pl.tw[2][(int)(((int64_t)kd * d) % D)];  // (cos, -sin)
      v = part ? -tw.y : tw.x;
    }
    Bt[e] = v;
  }
  const FastDiv fd = FastDiv::make(D);
  const int nitems = (KW + 1) * NDk;
  int ikw[NI], ikd[NI];
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    const int it = tid + q * BAND_NT;
    ikw[q] = it < nitems ? it / NDk : -1;
    ikd[q] = it < nitems ? it - (it / NDk) * NDk : 0;
  }
  const int units = H * a.nbc;
  const int nch = (W + BAND_ROWS_A - 1) / BAND_ROWS_A;
  const bool contig = a.sw == D;
  // (unit, chunk) sequence of this workgroup
  int u = (int)blockIdx.x, c = 0;
  if (u >= units) return;
  auto xbase = [&](int uu) {
    const int bcl = uu / H, hh = uu - bcl * H;
    return a.x + (int64_t)(a.bc0 + bcl) * a.sbc + (int64_t)hh * a.sh;
  };
  f32x4 pf[BAND_PF];
  ChunkSrc cs = chunk_src(xbase(u), a.sw, 0, W < BAND_ROWS_A ? W : BAND_ROWS_A, D);
  const int diag = a.diag;
  if (contig) chunk_load(pf, cs, tid);
  float2 Ac[NI], As[NI];
#pragma unroll
  for (int q = 0; q < NI; ++q) Ac[q] = As[q] = make_float2(0.f, 0.f);
  const int rbase = 16 * wv;  // this wave's 16 rows of the chunk
  for (;;) {
    const int w0 = c * BAND_ROWS_A;
    const int nr = (W - w0) < BAND_ROWS_A ? (W - w0) : BAND_ROWS_A;
    const float* xs = X;
    if (diag & 2)
      xs = X;
    else if (contig)
      xs = chunk_store(X, pf, cs, D, fd, tid);
    else
      chunk_copy_strided(X, P, cs, a.sw, D, fd, tid);
    __syncthreads();  // xs ready; every lane is past the previous chunk's W stage (Rb free)
    // next (unit, chunk): its loads fly while this chunk is computed
    int un = u, cn = c + 1;
    if (cn == nch) { cn = 0; un = u + (int)gridDim.x; }
    if (un < units) {
      const int w0n = cn * BAND_ROWS_A;
      cs = chunk_src(xbase(un), a.sw, w0n, (W - w0n) < BAND_ROWS_A ? (W - w0n) : BAND_ROWS_A, D);
      if (contig && !(diag & 1)) chunk_load(pf, cs, tid);
    }
    // D stage on the matrix cores: R(row, kd) = sum_d s_d cos + i sum_d t_d sin (folded over d, D - d)
    if (!(diag & 4)) {
      const float* row = xs + (rbase + l15) * P;
      f32x4 accc[NT2], accs[NT2];
#pragma unroll
      for (int nt = 0; nt < NT2; ++nt)
#pragma unroll
        for (int j = 0; j < 4; ++j) accc[nt][j] = accs[nt][j] = 0.f;
      for (int ks = 0; ks < KSd; ++ks) {
        const int d = 4 * ks + l4;
        const bool has = d < Ld;
        const bool pair = d >= 1 && 2 * d < D;
        const float xa = has ? row[d] : 0.f;
        const float xm = pair ? row[D - d] : 0.f;
        const float sv = xa + xm, tv = pair ? xm - xa : 0.f;
#pragma unroll
        for (int nt = 0; nt < NT2; ++nt) {
          const float* bt = Bt + ((nt * KSd + ks) * 2) * 64 + lane;
          accc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(sv, bt[0], accc[nt], 0, 0, 0);
          accs[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(tv, bt[64], accs[nt], 0, 0, 0);
        }
      }
      // lane holds rows rbase + 4 (l/16) + j of kd = 16 nt + l%16
#pragma unroll
      for (int nt = 0; nt < NT2; ++nt) {
        const int kd = 16 * nt + l15;
        if (kd < NDk)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            Rb[kd * (BAND_ROWS_A + 1) + rbase + 4 * l4 + j] = make_float2(accc[nt][j], accs[nt][j]);
      }
    }
    __syncthreads();  // Rb ready
    // W stage: per (kw >= 0, kd): Ac += R_w cos, As += R_w sin (theta = 2 pi kw w / W)
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (ikw[q] < 0 || (diag & 8)) continue;
      const int kw = ikw[q];
      const float2* Rk = Rb + ikd[q] * (BAND_ROWS_A + 1);
      int t = (int)(((int64_t)kw * w0) % W);
      float2 ac = Ac[q], as = As[q];
#pragma unroll 4
      for (int i = 0; i < nr; ++i) {
        const float2 r = Rk[i];
        const float2 tw = twW[t];
        ac.x = fmaf(r.x, tw.x, ac.x);
        ac.y = fmaf(r.y, tw.x, ac.y);
        as.x = fmaf(r.x, -tw.y, as.x);
        as.y = fmaf(r.y, -tw.y, as.y);
        t += kw;
        t = t >= W ? t - W : t;
      }
      Ac[q] = ac;
      As[q] = as;
    }
    if (c == nch - 1) {  // P(kw) = Ac - i As, P(-kw) = Ac + i As
      const int bcl = u / H, h = u - bcl * H, bc = a.bc0 + bcl;
      cf* Pb = a.P + ((int64_t)bc * H + h) * ncol;
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if (ikw[q] < 0) continue;
        const int kw = ikw[q], kd = ikd[q];
        Pb[(KW + kw) * NDk + kd] = mk(Ac[q].x + As[q].y, Ac[q].y - As[q].x);
        if (kw > 0) Pb[(KW - kw) * NDk + kd] = mk(Ac[q].x - As[q].y, Ac[q].y + As[q].x);
        Ac[q] = As[q] = make_float2(0.f, 0.f);
      }
    }
    if (un >= units) break;
    u = un;
    c = cn;
  }
}

// ----------------------------------------------------------------------------- pass B'
__global__ __launch_bounds__(BAND_NT) void k_band_mid(BandMidArgs) {
  const BandMidArgs& a = kargs<BandMidArgs>();
  __shared__ float4 red[3][64];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, ncol = a.g.ncol;
  const int kh = (int)blockIdx.y, bcl = (int)blockIdx.z, bc = a.bc0 + bcl;
  const int col = (int)blockIdx.x * 64 + lane;
  const bool live = col < ncol;
  const cf* Pc = a.P + (int64_t)bc * H * ncol + (live ? col : 0);
  const cf* twH = a.pl.tw[0];
  // Q(kh) = sum_h P_h e^{-i theta}: Ac = sum P cos, As = sum P sin; waves split h
  float2 ac = make_float2(0.f, 0.f), as = make_float2(0.f, 0.f);
  int t = (int)(((int64_t)kh * wv) % H);
  const int step = (int)(((int64_t)kh * 4) % H);
  for (int hh = wv; hh < H; hh += 4) {
    const float2 p = ld2(Pc + (int64_t)hh * ncol);
    const float2 tw = ld2(twH + t);  // uniform: (cos, -sin)
    ac.x = fmaf(p.x, tw.x, ac.x);
    ac.y = fmaf(p.y, tw.x, ac.y);
    as.x = fmaf(p.x, -tw.y, as.x);
    as.y = fmaf(p.y, -tw.y, as.y);
    t += step;
    t = t >= H ? t - H : t;
  }
  if (wv > 0) red[wv - 1][lane] = make_float4(ac.x, ac.y, as.x, as.y);
  __syncthreads();
  if (wv != 0) return;
  for (int j = 0; j < 3; ++j) {
    const float4 r = red[j][lane];
    ac.x += r.x; ac.y += r.y; as.x += r.z; as.y += r.w;
  }
  const int lb = a.cofs + bcl, s = lb / a.C, chan = lb - s * a.C;
  const tb_sample_ops& so = a.ops.s[s];
  if (live) {
    const int jw = col / NDk, kd = col - jw * NDk;
    const int kw = (jw - KW + W) % W;
    const FreqCol fc = freq_col(kw, kd, W, D);
    cf qp = apply_ops(so, chan, mk(ac.x + as.y, ac.y - as.x), fc, kh, H);
    float4 o;
    if (kh == 0) {
      o = make_float4(qp.x, qp.y, 0.f, 0.f);
    } else {
      const cf qm = apply_ops(so, chan, mk(ac.x - as.y, ac.y + as.x), fc, H - kh, H);
      o = make_float4(qp.x + qm.x, qp.y + qm.y, qp.x - qm.x, qp.y - qm.y);
    }
    a.AB[((int64_t)bc * (a.g.KH + 1) + kh) * ncol + col] = o;
  }
  // the out-of-box spike points: the program applied to a coefficient the low-pass zeroed
  if (blockIdx.x == 0 && kh == 0 && lane < BAND_MAX_PTS) {
    const BandSamplePts& sp = a.sp[s];
    cf c = mk(0.f, 0.f);
    if (lane < sp.n) {
      const BandPt p = sp.p[lane];
      c = apply_ops(so, chan, mk(0.f, 0.f), freq_col(p.kw, p.kd, W, D), p.kh, H);
    }
    a.pts[(int64_t)bc * BAND_MAX_PTS + lane] = c;
  }
}

// ----------------------------------------------------------------------------- pass C'
// Per (bc, h) slab, all on the matrix cores after a small VALU prologue:
//   Z_h(kw, kd)  = A_0 + sum_kh>=1 (A cos + i B sin)           (VALU; AB from pass B')
//   V^T(v, w)    = M2T(v, k) . CS(k, w)                        (MFMA 32x32x2; v = 2 kd + re/im and
//                  two rows per out-of-box point, k = (kw, cos/sin) terms; w on the lane)
//   Y^T(n, w)    = B^T(n, v) . V^T(v, w)                       (MFMA, V^T straight from the
//                  accumulators: the k order of each step is the accumulator's row pair
//                  (rho(s), rho(s) + 4), the same permutation indexes the B table)
// so each lane ends with 4 consecutive output columns of one image row: 16-B stores.
__device__ __forceinline__ int acc_row(int s) { return (s & 3) + 8 * (s >> 2); }  // rho(s)

template <int VT>  // 32-row tiles of V (2 (NDk + points) <= 32 VT)
__global__ __launch_bounds__(BAND_NT) void k_band_inv(BandInvArgs) {
  const BandInvArgs& a = kargs<BandInvArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[2 * BAND_NT / 64];
  const int tid = (int)threadIdx.x, lane = tid & 63, hl = lane >> 5, l31 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, KH = a.g.KH, ncol = a.g.ncol, NCOL = a.g.NCOL;
  const int npm = a.g.KS - NDk;        // point rows of the launch (max over its samples)
  const int KV = KW + 1 + npm;         // k-steps of the V product
  const int MP = 2 * KV + 1;           // M2T pitch
  const BandInvCarve cv = band_inv_carve(a.g, W);
  float* Bimg = reinterpret_cast<float*>(smem + cv.bimg);  // [32 VT][NCOL]
  float* M2T = reinterpret_cast<float*>(smem + cv.va);     // [32 VT][MP]
  float2* Zb = reinterpret_cast<float2*>(smem + cv.zb);    // [ncol]
  float2* twW = reinterpret_cast<float2*>(smem + cv.tww);  // (cos, -sin)(2 pi t / W)
  const cf* twD = a.pl.tw[2];
  for (int t = tid; t < W; t += BAND_NT) twW[t] = ld2(a.pl.tw[1] + t);
  // synthesis table rows v: 2k -> cos(2 pi kd_k n / D), 2k + 1 -> -sin; 0 for n >= D and unused rows
  for (int e = tid; e < 32 * VT * NCOL; e += BAND_NT) {
    const int r = e / NCOL, n = e - r * NCOL, k = r >> 1;
    float v = 0.f;
    if (k < NDk && n < D) {
      const cf tw = twD[(int)(((int64_t)k * n) % D)];
      v = (r & 1) ? tw.y : tw.x;
    }
    Bimg[e] = v;
  }
  const int units = H * a.nbc;
  const int ntw = (W + 31) / 32;     // 32-row tiles of the slab
  const int ntn = NCOL / 32;         // 32-column tiles of the output row
  const int ycols = D + a.ypad;
  const int diag = a.diag;
  int cur_s = -1;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int u = (int)blockIdx.x; u < units; u += (int)gridDim.x) {
    const int bcl = u / H, h = u - bcl * H, bc = a.bc0 + bcl;
    const int s = (a.cofs + bcl) / a.C;
    const BandSamplePts& sp = a.sp[s];
    __syncthreads();  // the previous unit is done with Zb / M2T / the point rows of Bimg
    if (s != cur_s && npm > 0) {
      for (int e = tid; e < 2 * npm * NCOL; e += BAND_NT) {
        const int r = e / NCOL, n = e - r * NCOL, j = r >> 1;
        float v = 0.f;
        if (j < sp.n && n < D) {
          const cf tw = twD[(int)(((int64_t)sp.p[j].kd * n) % D)];
          v = (r & 1) ? tw.y : tw.x;
        }
        Bimg[(2 * NDk + r) * NCOL + n] = v;
      }
    }
    cur_s = s;
    // Z_h(col) = A_0 + sum_kh>=1 (A cos + i B sin), theta = 2 pi kh h / H; loads issued 4 at a time
    const float4* ABb = a.AB + (int64_t)bc * (KH + 1) * ncol;
    for (int col = (diag & 1) ? ncol : tid; col < ncol; col += BAND_NT) {
      const float4 a0 = ABb[col];
      float zx = a0.x, zy = a0.y;
      int t = 0;
      for (int k0 = 1; k0 <= KH; k0 += 4) {
        float4 ab[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (k0 + q <= KH) ab[q] = ABb[(int64_t)(k0 + q) * ncol + col];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (k0 + q > KH) break;
          t += h;
          t = t >= H ? t - H : t;
          const cf tw = a.pl.tw[0][t];  // (cos, -sin)
          zx = fmaf(ab[q].x, tw.x, fmaf(ab[q].w, tw.y, zx));   // - B.y sin
          zy = fmaf(ab[q].y, tw.x, fmaf(-ab[q].z, tw.y, zy));  // + B.x sin
        }
      }
      Zb[col] = make_float2(zx, zy);
    }
    // the sample's point coefficients rotated to this slab: ph_j = c_j e^{+2 pi i kh_j h / H} wt / N
    float2 ph[BAND_MAX_PTS];
#pragma unroll
    for (int j = 0; j < BAND_MAX_PTS; ++j) {
      ph[j] = make_float2(0.f, 0.f);
      if (j < sp.n && j < npm) {
        const cf c = a.pts[(int64_t)bc * BAND_MAX_PTS + j];
        const cf tw = a.pl.tw[0][(int)(((int64_t)sp.p[j].kh * h) % H)];
        const float wt = ((sp.p[j].kd == 0 || 2 * sp.p[j].kd == D) ? 1.f : 2.f) * a.scale;
        ph[j] = make_float2((c.x * tw.x + c.y * tw.y) * wt, (c.y * tw.x - c.x * tw.y) * wt);
      }
    }
    __syncthreads();
    // M2T(v, k): Vr = sum (Ar cos - Bi sin), Vi = sum (Ai cos + Br sin) over kw; points: ph e^{+i phi}
    for (int e = (diag & 2) ? 32 * VT * 2 * KV : tid; e < 32 * VT * 2 * KV; e += BAND_NT) {
      const int r = e / (2 * KV), k = e - r * (2 * KV);
      const int ks = k >> 1, sn = k & 1, im = r & 1, kd = r >> 1;
      float v = 0.f;
      if (kd < NDk) {
        if (ks <= KW) {
          const float2 zp = Zb[(KW + ks) * NDk + kd];
          float2 A = zp, B = make_float2(0.f, 0.f);
          if (ks > 0) {
            const float2 zm = Zb[(KW - ks) * NDk + kd];
            A = make_float2(zp.x + zm.x, zp.y + zm.y);
            B = make_float2(zp.x - zm.x, zp.y - zm.y);
          }
          const float wt = ((kd == 0 || 2 * kd == D) ? 1.f : 2.f) * a.scale;
          v = (im ? (sn ? B.x : A.y) : (sn ? -B.y : A.x)) * wt;
        }
      } else if (kd - NDk < npm) {
        const int j = kd - NDk;
        if (ks == KW + 1 + j) {
          float2 c = make_float2(0.f, 0.f);
#pragma unroll
          for (int jj = 0; jj < BAND_MAX_PTS; ++jj)
            if (jj == j) c = ph[jj];
          v = im ? (sn ? c.x : c.y) : (sn ? -c.y : c.x);
        }
      }
      M2T[r * MP + k] = v;
    }
    __syncthreads();
    const float* afr = M2T + l31 * MP + hl;  // A fragment of k-step ks, tile vt: afr[32 vt MP + 2 ks]
    float* yb = a.y + (int64_t)bc * a.sbc + (int64_t)h * a.sh;
    const bool vec = ((a.sw & 3) == 0) && ((reinterpret_cast<uintptr_t>(yb) & 15) == 0);
    for (int tw_ = wv; tw_ < ntw; tw_ += 4) {
      const int w = 32 * tw_ + l31;
      const bool wok = w < W;
      const int wm = w % W;
      // V^T(:, w) for this lane's row w
      f32x16 vacc[VT];
#pragma unroll
      for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int j = 0; j < 16; ++j) vacc[vt][j] = 0.f;
      int t = 0;
      for (int ks = 0; ks <= ((diag & 4) ? -1 : KW); ++ks) {
        const float2 c = twW[t];
        const float b = hl ? -c.y : c.x;
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
          vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(afr[32 * vt * MP + 2 * ks], b, vacc[vt], 0, 0, 0);
        t += wm;
        t = t >= W ? t - W : t;
      }
      for (int j = 0; j < npm; ++j) {
        const int kw = j < sp.n ? sp.p[j].kw : 0;
        const float2 c = twW[(int)(((int64_t)kw * wm) % W)];
        const float b = hl ? -c.y : c.x;
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
          vacc[vt] = __builtin_amdgcn_mfma_f32_32x32x2f32(afr[32 * vt * MP + 2 * (KW + 1 + j)], b, vacc[vt], 0, 0, 0);
      }
      float* yr = yb + (int64_t)w * a.sw;
      for (int nt = 0; nt < ntn; ++nt) {
        f32x16 y;
#pragma unroll
        for (int j = 0; j < 16; ++j) y[j] = 0.f;
        const float* bb = Bimg + (4 * hl) * NCOL + nt * 32 + l31;
        if (!(diag & 8))
#pragma unroll
          for (int vt = 0; vt < VT; ++vt)
#pragma unroll
            for (int sI = 0; sI < 16; ++sI)
              y = __builtin_amdgcn_mfma_f32_32x32x2f32(bb[(32 * vt + acc_row(sI)) * NCOL], vacc[vt][sI], y, 0, 0, 0);
        if (!wok || (diag & 16)) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n0 = nt * 32 + 8 * g + 4 * hl;
          const float v0 = y[4 * g], v1 = y[4 * g + 1], v2 = y[4 * g + 2], v3 = y[4 * g + 3];
          if (vec && n0 + 4 <= ycols) {
            *reinterpret_cast<float4*>(yr + n0) = make_float4(v0, v1, v2, v3);
          } else {
            const float vv[4] = {v0, v1, v2, v3};
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (n0 + q < ycols) yr[n0 + q] = vv[q];
          }
          const float vv[4] = {v0, v1, v2, v3};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (n0 + q < D) {
              lo = fminf(lo, vv[q]);
              hi = fmaxf(hi, vv[q]);
            }
        }
      }
    }
    // flush the running min/max when the next unit belongs to another sample (or there is none)
    const int un = u + (int)gridDim.x;
    const int b = bc / a.C;
    if (a.mm && (un >= units || (a.bc0 + un / H) / a.C != b)) {
      block_minmax_atomic<BAND_NT>(lo, hi, red, a.mm + 2 * b);
      lo = 3.402823466e38f;
      hi = -3.402823466e38f;
    }
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

int band_grid(int units, size_t lds, int ncu) {
  int per_cu = (int)(163840 / (lds ? lds : 1));
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  const int g = ncu * per_cu;
  return units < g ? units : g;
}

template <int NT2, int NI>
hipError_t launch_fwd_t(const BandFwdArgs& a, size_t lds, int ncu, hipStream_t st) {
  auto kern = k_band_fwd<NT2, NI>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int units = a.pl.H * a.nbc;
  hipLaunchKernelGGL(kern, dim3(band_grid(units, lds, ncu)), dim3(BAND_NT), lds, st, a);
  return hipGetLastError();
}

template <int NT2>
hipError_t launch_fwd_nt(const BandFwdArgs& a, size_t lds, int ncu, hipStream_t st) {
  const int items = (a.g.KW + 1) * a.g.NDk;
  if (items <= BAND_NT) return launch_fwd_t<NT2, 1>(a, lds, ncu, st);
  if (items <= 2 * BAND_NT) return launch_fwd_t<NT2, 2>(a, lds, ncu, st);
  return launch_fwd_t<NT2, 4>(a, lds, ncu, st);
}

template <int VT>
hipError_t launch_inv_t(const BandInvArgs& a, int ncu, hipStream_t st) {
  const size_t lds = band_inv_carve(a.g, a.pl.W).total;
  auto kern = k_band_inv<VT>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int units = a.pl.H * a.nbc;
  hipLaunchKernelGGL(kern, dim3(band_grid(units, lds, ncu)), dim3(BAND_NT), lds, st, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_band_fwd(const BandFwdArgs& a, int ncu, hipStream_t st) {
  const size_t lds = band_lds_fwd(a.g, a.pl.W, a.pl.D);
  return a.g.NDk <= 16 ? launch_fwd_nt<1>(a, lds, ncu, st) : launch_fwd_nt<2>(a, lds, ncu, st);
}

hipError_t launch_band_mid(const BandMidArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_band_mid, dim3((a.g.ncol + 63) / 64, a.g.KH + 1, a.nbc), dim3(BAND_NT), 0, st, a);
  return hipGetLastError();
}



hipError_t launch_band_inv(const BandInvArgs& a, int ncu, hipStream_t st) {
  return 2 * a.g.KS <= 32 ? launch_inv_t<1>(a, ncu, st) : launch_inv_t<2>(a, ncu, st);
}

hipError_t launch_copy_pad(const CopyArgs& a, hipStream_t st) {
  const int units = a.H * a.nbc;
  const int g = units < 2048 ? units : 2048;
  hipLaunchKernelGGL(k_copy_pad, dim3(g), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace tb
