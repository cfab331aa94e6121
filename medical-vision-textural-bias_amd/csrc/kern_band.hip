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
// Copy n image rows (global rows g0.., row pitch sw, D floats each) into LDS rows 0.. of pitch
// P.  Contiguous rows (sw == D) stream as 16-B lanes from the 16-B-aligned address at or below
// the first element; the few out-of-range elements of the first/last vector are dropped.
template <int U>
__device__ __forceinline__ void band_load_rows(float* xs, int P, const float* __restrict__ xb, int64_t sw, int g0,
                                               int n, int D, const FastDiv& fd, int tid) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const float* src = xb + (int64_t)g0 * sw;
  const int total = n * D;
  if (sw == D) {
    const int off = (int)((reinterpret_cast<uintptr_t>(src) >> 2) & 3);
    const f32x4* s4 = reinterpret_cast<const f32x4*>(src - off);
    const int nq = (total + off + 3) >> 2;
    const bool odd = (D & 1) != 0;
    for (int q0 = tid; q0 < nq; q0 += BAND_NT * U) {
      f32x4 v[U];  // U independent 16-B loads in flight per lane before the first LDS store
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * BAND_NT;
        if (q < nq) v[u] = __builtin_nontemporal_load(s4 + q);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * BAND_NT;
        if (q >= nq) break;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = 4 * q + k - off;
          if (e >= 0 && e < total) xs[odd ? e : e + fd.div(e)] = v[u][k];
        }
      }
    }
  } else {
    for (int e0 = tid; e0 < total; e0 += BAND_NT * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * BAND_NT;
        if (e < total) {
          const int r = fd.div(e);
          v[u] = src[(int64_t)r * sw + (e - r * D)];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * BAND_NT;
        if (e < total) {
          const int r = fd.div(e);
          xs[r * P + (e - r * D)] = v[u];
        }
      }
    }
  }
}

// NK: kd values per wave (4 waves: NDk <= 4 NK); NI: stage-W items per thread ((KW+1) NDk <= 256 NI)
template <int NK, int NI>
__global__ __launch_bounds__(BAND_NT) void k_band_fwd(BandFwdArgs) {
  const BandFwdArgs& a = kargs<BandFwdArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, ncol = a.g.ncol;
  const int P = (D & 1) ? D : D + 1;
  float* xs = reinterpret_cast<float*>(smem);
  float2* Rb = reinterpret_cast<float2*>(xs + BAND_ROWS_A * P);  // [kd][65]
  float2* twW = Rb + NDk * (BAND_ROWS_A + 1);                     // (cos, -sin)(2 pi t / W)
  for (int t = tid; t < W; t += BAND_NT) twW[t] = ld2(a.pl.tw[1] + t);
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
  const int kd0 = wv * NK;
  const bool dwave = kd0 < NDk;  // this wave owns at least one kd
  const int npair = (D - 1) / 2;  // d in [1, npair] pairs with D - d
  // twiddles are wave-uniform: read them through the constant address space so they arrive by
  // scalar loads into SGPRs (a generic pointer gets per-lane vector loads of the same bytes)
  typedef const __attribute__((address_space(4))) float cfloat;
  const cfloat* tdf = (const cfloat*)(a.tdf + kd0);  // (cos, sin) pairs
  const int NKP = a.NKP;
  for (int u = (int)blockIdx.x; u < units; u += (int)gridDim.x) {
    const int bcl = u / H, h = u - bcl * H, bc = a.bc0 + bcl;
    const float* __restrict__ xb = a.x + (int64_t)bc * a.sbc + (int64_t)h * a.sh;
    float2 Ac[NI], As[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) Ac[q] = As[q] = make_float2(0.f, 0.f);
    for (int c = 0; c < nch; ++c) {
      const int w0 = c * BAND_ROWS_A;
      const int nr = (W - w0) < BAND_ROWS_A ? (W - w0) : BAND_ROWS_A;
      __syncthreads();  // the previous chunk's readers of xs / Rb are done
      band_load_rows<10>(xs, P, xb, a.sw, w0, nr, D, fd, tid);
      __syncthreads();
      // D stage: lane = row, this wave's kd group; X(kd) = x0 + sum_d s_d cos - i t_d sin
      if (dwave) {
        const float* row = xs + lane * P;
        float re[NK], im[NK];
        const float x0 = row[0];
#pragma unroll
        for (int k = 0; k < NK; ++k) { re[k] = x0; im[k] = 0.f; }
#pragma unroll 4
        for (int d = 1; d <= npair; ++d) {
          const float xa = row[d], xm = row[D - d];
          const float s = xa + xm, t = xm - xa;
          const cfloat* tt = tdf + 2 * d * NKP;
#pragma unroll
          for (int k = 0; k < NK; ++k) {
            re[k] = fmaf(s, tt[2 * k], re[k]);
            im[k] = fmaf(t, tt[2 * k + 1], im[k]);
          }
        }
        if ((D & 1) == 0) {  // d = D/2 has no partner: cos = (-1)^kd, sin = 0
          const float xh = row[D / 2];
          const cfloat* tt = tdf + 2 * (D / 2) * NKP;
#pragma unroll
          for (int k = 0; k < NK; ++k) re[k] = fmaf(xh, tt[2 * k], re[k]);
        }
#pragma unroll
        for (int k = 0; k < NK; ++k)
          if (kd0 + k < NDk) Rb[(kd0 + k) * (BAND_ROWS_A + 1) + lane] = make_float2(re[k], im[k]);
      }
      __syncthreads();
      // W stage: per (kw >= 0, kd): Ac += R_w cos, As += R_w sin (theta = 2 pi kw w / W)
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if (ikw[q] < 0) continue;
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
    }
    // P(kw) = Ac - i As, P(-kw) = Ac + i As
    cf* Pb = a.P + ((int64_t)bc * H + h) * ncol;
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (ikw[q] < 0) continue;
      const int kw = ikw[q], kd = ikd[q];
      Pb[(KW + kw) * NDk + kd] = mk(Ac[q].x + As[q].y, Ac[q].y - As[q].x);
      if (kw > 0) Pb[(KW - kw) * NDk + kd] = mk(Ac[q].x - As[q].y, Ac[q].y + As[q].x);
    }
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
__global__ __launch_bounds__(BAND_NT) void k_band_inv(BandInvArgs) {
  const BandInvArgs& a = kargs<BandInvArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[2 * BAND_NT / 64];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int NDk = a.g.NDk, KW = a.g.KW, KH = a.g.KH, ncol = a.g.ncol, KS = a.g.KS, NCOL = a.g.NCOL;
  const int KC2 = 2 * KS, VP = KC2 + 1;
  const BandInvCarve cv = band_inv_carve(a.g, W);
  float* Bimg = reinterpret_cast<float*>(smem + cv.bimg);    // [KC2][NCOL]
  float* Va = reinterpret_cast<float*>(smem + cv.va);        // [128][VP]
  float2* Zb = reinterpret_cast<float2*>(smem + cv.zb);      // [ncol]
  float4* AwBw = reinterpret_cast<float4*>(smem + cv.awbw);  // [KW+1][NDk]
  float2* twW = reinterpret_cast<float2*>(smem + cv.tww);    // (cos, -sin)(2 pi t / W)
  const cf* twD = a.pl.tw[2];
  for (int t = tid; t < W; t += BAND_NT) twW[t] = ld2(a.pl.tw[1] + t);
  for (int t = tid; t < BAND_ROWS_C * VP; t += BAND_NT) Va[t] = 0.f;
  // band rows of the D-synthesis table: B[2k][n] = cos(2 pi k n / D), B[2k+1][n] = -sin, 0 for n >= D
  for (int e = tid; e < 2 * NDk * NCOL; e += BAND_NT) {
    const int r = e / NCOL, n = e - r * NCOL, k = r >> 1;
    float v = 0.f;
    if (n < D) {
      const cf tw = twD[(int)(((int64_t)k * n) % D)];
      v = (r & 1) ? tw.y : tw.x;
    }
    Bimg[e] = v;
  }
  const int units = H * a.nbc;
  const int npt_rows = KS - NDk;  // point columns of the table (the launch's max points)
  int cur_s = -1;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  const int ncnk = (W + BAND_ROWS_C - 1) / BAND_ROWS_C;
  const int ntile = NCOL / 32;
  const int ycols = D + a.ypad;
  for (int u = (int)blockIdx.x; u < units; u += (int)gridDim.x) {
    const int bcl = u / H, h = u - bcl * H, bc = a.bc0 + bcl;
    const int lb = a.cofs + bcl, s = lb / a.C;
    const BandSamplePts& sp = a.sp[s];
    __syncthreads();  // previous unit done with Zb / AwBw / Va / Bimg
    if (s != cur_s && npt_rows > 0) {  // the sample's point rows of the table
      for (int e = tid; e < 2 * npt_rows * NCOL; e += BAND_NT) {
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
    // Z_h(col) = A_0 + sum_kh>=1 (A cos + i B sin), theta = 2 pi kh h / H
    const float4* ABb = a.AB + (int64_t)bc * (KH + 1) * ncol;
    for (int col = tid; col < ncol; col += BAND_NT) {
      const float4 a0 = ABb[col];
      float zx = a0.x, zy = a0.y;
      int t = 0;
      for (int k = 1; k <= KH; ++k) {
        t += h;
        t = t >= H ? t - H : t;
        const float4 ab = ABb[(int64_t)k * ncol + col];
        const cf tw = a.pl.tw[0][t];  // (cos, -sin)
        zx = fmaf(ab.x, tw.x, fmaf(ab.w, tw.y, zx));   // - B.y sin
        zy = fmaf(ab.y, tw.x, fmaf(-ab.z, tw.y, zy));  // + B.x sin
      }
      Zb[col] = make_float2(zx, zy);
    }
    __syncthreads();
    // W-pair sums: A_kw = Z(kw) + Z(-kw), B_kw = Z(kw) - Z(-kw)
    for (int it = tid; it < (KW + 1) * NDk; it += BAND_NT) {
      const int kw = it / NDk, kd = it - kw * NDk;
      const float2 zp = Zb[(KW + kw) * NDk + kd];
      if (kw == 0) {
        AwBw[it] = make_float4(zp.x, zp.y, 0.f, 0.f);
      } else {
        const float2 zm = Zb[(KW - kw) * NDk + kd];
        AwBw[it] = make_float4(zp.x + zm.x, zp.y + zm.y, zp.x - zm.x, zp.y - zm.y);
      }
    }
    // the sample's point coefficients, rotated to this slab's h: c e^{+2 pi i kh_p h / H} wt / N
    float2 ph[BAND_MAX_PTS];
#pragma unroll
    for (int j = 0; j < BAND_MAX_PTS; ++j) {
      ph[j] = make_float2(0.f, 0.f);
      if (j < sp.n && j < npt_rows) {
        const cf c = a.pts[(int64_t)bc * BAND_MAX_PTS + j];
        const cf tw = a.pl.tw[0][(int)(((int64_t)sp.p[j].kh * h) % H)];
        const float wt = ((sp.p[j].kd == 0 || 2 * sp.p[j].kd == D) ? 1.f : 2.f) * a.scale;
        // c * conj(tw) = c e^{+i theta}  (tw = e^{-i theta})
        ph[j] = make_float2((c.x * tw.x + c.y * tw.y) * wt, (c.y * tw.x - c.x * tw.y) * wt);
      }
    }
    __syncthreads();
    float* yb = a.y + (int64_t)bc * a.sbc + (int64_t)h * a.sh;
    for (int cc = 0; cc < ncnk; ++cc) {
      const int w0 = cc * BAND_ROWS_C;
      const int nr = (W - w0) < BAND_ROWS_C ? (W - w0) : BAND_ROWS_C;
      if (cc > 0) __syncthreads();  // the previous chunk's MFMA reads of Va are done
      // V_w(kd) = sum_kw>=0 (A cos + i B sin), theta = 2 pi kw w / W; scaled by wt(kd) / N
      for (int it = tid; it < nr * NDk; it += BAND_NT) {
        const int i = it / NDk, kd = it - i * NDk;
        const int w = w0 + i;
        float sx = 0.f, sy = 0.f;
        int t = 0;
        const float4* ab = AwBw + kd;
        for (int kw = 0; kw <= KW; ++kw) {
          const float4 v = ab[kw * NDk];
          const float2 tw = twW[t];  // (cos, -sin)
          sx = fmaf(v.x, tw.x, fmaf(v.w, tw.y, sx));
          sy = fmaf(v.y, tw.x, fmaf(-v.z, tw.y, sy));
          t += w;
          t = t >= W ? t - W : t;
        }
        const float wt = ((kd == 0 || 2 * kd == D) ? 1.f : 2.f) * a.scale;
        Va[i * VP + 2 * kd] = sx * wt;
        Va[i * VP + 2 * kd + 1] = sy * wt;
      }
      // point columns: ph_j e^{+2 pi i kw_p w / W}
      for (int it = tid; it < nr * npt_rows; it += BAND_NT) {
        const int i = it / npt_rows, j = it - i * npt_rows;
        float vx = 0.f, vy = 0.f;
        if (j < sp.n) {
          const int w = w0 + i;
          const float2 tw = twW[(int)(((int64_t)sp.p[j].kw * w) % W)];
          float2 c = make_float2(0.f, 0.f);
#pragma unroll
          for (int jj = 0; jj < BAND_MAX_PTS; ++jj)
            if (jj == j) c = ph[jj];
          vx = c.x * tw.x + c.y * tw.y;
          vy = c.y * tw.x - c.x * tw.y;
        }
        Va[i * VP + 2 * (NDk + j)] = vx;
        Va[i * VP + 2 * (NDk + j) + 1] = vy;
      }
      __syncthreads();
      // D synthesis on the matrix cores: y[m][n] = sum_k Va[m][k] B[k][n]; wave = 32-row tile
      const int mrow0 = wv * 32;
      if (mrow0 < nr) {
        const float* va = Va + (mrow0 + (lane & 31)) * VP + (lane >> 5);
        for (int nt = 0; nt < ntile; ++nt) {
          f32x16 acc;
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[j] = 0.f;
          const float* bb = Bimg + (lane >> 5) * NCOL + nt * 32 + (lane & 31);
          for (int ks = 0; ks < KS; ++ks)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(va[2 * ks], bb[2 * ks * NCOL], acc, 0, 0, 0);
          const int n = nt * 32 + (lane & 31);
          if (n < ycols) {
            const bool real = n < D;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const int m = (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
              if (mrow0 + m < nr) {
                const float v = acc[j];
                yb[(int64_t)(w0 + mrow0 + m) * a.sw + n] = v;
                if (real) {
                  lo = fminf(lo, v);
                  hi = fmaxf(hi, v);
                }
              }
            }
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

template <int NK, int NI>
hipError_t launch_fwd_t(const BandFwdArgs& a, size_t lds, int ncu, hipStream_t st) {
  auto kern = k_band_fwd<NK, NI>;
  hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int units = a.pl.H * a.nbc;
  hipLaunchKernelGGL(kern, dim3(band_grid(units, lds, ncu)), dim3(BAND_NT), lds, st, a);
  return hipGetLastError();
}

template <int NK>
hipError_t launch_fwd_nk(const BandFwdArgs& a, size_t lds, int ncu, hipStream_t st) {
  const int items = (a.g.KW + 1) * a.g.NDk;
  if (items <= BAND_NT) return launch_fwd_t<NK, 1>(a, lds, ncu, st);
  if (items <= 2 * BAND_NT) return launch_fwd_t<NK, 2>(a, lds, ncu, st);
  return launch_fwd_t<NK, 4>(a, lds, ncu, st);
}

}  // namespace

hipError_t launch_band_fwd(const BandFwdArgs& a, int ncu, hipStream_t st) {
  const size_t lds = band_lds_fwd(a.g, a.pl.W, a.pl.D);
  const int nk = (a.g.NDk + 3) / 4;
  if (nk <= 1) return launch_fwd_nk<1>(a, lds, ncu, st);
  if (nk <= 2) return launch_fwd_nk<2>(a, lds, ncu, st);
  if (nk <= 4) return launch_fwd_nk<4>(a, lds, ncu, st);
  return launch_fwd_nk<8>(a, lds, ncu, st);
}

hipError_t launch_band_mid(const BandMidArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_band_mid, dim3((a.g.ncol + 63) / 64, a.g.KH + 1, a.nbc), dim3(BAND_NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_band_inv(const BandInvArgs& a, int ncu, hipStream_t st) {
  const size_t lds = band_inv_carve(a.g, a.pl.W).total;
  hipError_t e = allow_lds(k_band_inv, lds);
  if (e != hipSuccess) return e;
  const int units = a.pl.H * a.nbc;
  hipLaunchKernelGGL(k_band_inv, dim3(band_grid(units, lds, ncu)), dim3(BAND_NT), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_copy_pad(const CopyArgs& a, hipStream_t st) {
  const int units = a.H * a.nbc;
  const int g = units < 2048 ? units : 2048;
  hipLaunchKernelGGL(k_copy_pad, dim3(g), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace tb
