// kern_point.hip -- closed-form route for spike-only programs (point.h).
//
// Reference: RandPlaneWaves_ellipsoid.__call__ (source_code/filters_and_operators.py:370-393) and
// KSpaceSpikeNoise._set_spike (:966-983): FFT, set |K(f)| = exp(intensity) at one location with the
// phase kept, inverse FFT, `.real`.  Only K(f_j) is needed, so the spectrum is never formed:
//   k_point_dft    one workgroup per (bc, h) slab: S_j(w) = sum_d x[w][d] e^{-2 pi i kd_j d / D} per
//                  row (one wave per row, lane = d), K_slab,j = e^{-2 pi i kh_j h / H} sum_w
//                  e^{-2 pi i kw_j w / W} S_j(w)  ->  part[bc][h][j] (float64)
//   k_point_delta  one wave per bc: K_j = sum_h part, Delta_j / N = (target_j(K_j) - K_j) / N
//   k_point_apply  one workgroup per slab: y[w][d] = x[w][d] + sum_j Re(R_j(w) e^{2 pi i kd_j d / D}),
//                  R_j(w) = Delta_j / N e^{2 pi i (kh_j h / H + kw_j w / W)}; zero D-padding; per-sample
//                  min/max keys (the salt-and-pepper MIN/MAX of a chain that continues with S&P)
// Algorithmic bytes: 4 B per voxel (dft) + 4 B in and 4 B (+ padding) out (apply).
#include "point.h"

#include <map>
#include <mutex>

namespace tb {

namespace {

// The spikes of (sample, channel) bcl, as LDS ints: n, then per spike (kh, kw, kd, op slot).  Filled
// by one thread (the op program lives in the kernarg segment; a per-thread copy with dynamic
// indexing would sit in scratch).
constexpr int PT_ACT = 1 + 4 * TB_MAX_OPS;
__device__ __forceinline__ void point_active(const PointArgs& a, int bcl, int* act) {
  if (threadIdx.x == 0) {
    const int s = bcl / a.C, c = bcl - s * a.C;
    const tb_sample_ops& so = a.ops.s[s];
    int n = 0;
    for (int o = 0; o < so.n; ++o) {
      const tb_op& op = so.op[o];
      if (op.chan >= 0 && op.chan != c) continue;
      act[1 + 4 * n] = op.i[0];
      act[2 + 4 * n] = op.i[1];
      act[3 + 4 * n] = op.i[2];
      act[4 + 4 * n] = o;
      ++n;
    }
    act[0] = n;
  }
  __syncthreads();
}

// e^{sgn 2 pi i m / n}, 0 <= m < n (float: the argument 2 m / n is rounded once)
__device__ __forceinline__ float2 cis_f(int m, int n, float sgn) {
  float s, c;
  sincospif(2.f * (float)m / (float)n, &s, &c);
  return make_float2(c, sgn * s);
}

__device__ __forceinline__ int mulmod(int a, int b, int n) { return (int)(((int64_t)a * b) % n); }

__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

}  // namespace

// Work item = a quad: 4 consecutive columns d0 .. d0 + 3 of one row (h, w); a volume-channel's quads
// are numbered row-major over (h, w, d0) and split into `parts` contiguous ranges, one per workgroup
// (2,048 workgroups a launch, each ~9 rounds of PT_QU quads per thread: one slab per workgroup left
// 1,920 short-lived workgroups and a second, nearly empty round of them).  Consecutive lanes take
// consecutive quads (coalesced); a thread issues all loads of a round before using them.
constexpr int PT_QU = 4;

// A whole quad is one 16-B load even where the row is only dword aligned (the 155-column BraTS rows):
// gfx950's global loads take dword-aligned dwordx4 addresses, and 64 lanes still sweep ~1 KB of
// consecutive bytes.  The partial last quad of a row loads the row's last 4 floats and shifts them
// down with selects: no branch, so no lane's tail forces a wait on the loads already in flight
// (a divergent scalar tail path made the compiler drain vmcnt at every row end).  D >= 4.
typedef float f32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ void load_quad(const float* row, int d0, int D, bool ok, float (&v)[4]) {
  const int dl = d0 + 4 <= D ? d0 : D - 4, sh = ok ? d0 - dl : 4;  // sh 4: nothing
#if TB_NT_LOADS  // (the builtin directly: ld_stream's template parameter would drop the 4-B alignment)
  const f32x4_a4 q = __builtin_nontemporal_load(reinterpret_cast<const f32x4_a4*>(row + dl));
#else
  const f32x4_a4 q = *reinterpret_cast<const f32x4_a4*>(row + dl);
#endif
  const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float t = 0.f;
#pragma unroll
    for (int s = 0; s + j < 4; ++s) t = sh == s ? e[j + s] : t;
    v[j] = t;
  }
}

// per-axis twiddle tables of the active spikes: along D quad-major, tD[(k * 4 + j) * NQ + q] =
// e^{sgn 2 pi i f_k,d (4q + j) / D} (zero for 4q + j >= D), so the lanes of a wave (consecutive quads)
// read consecutive entries; tW[k][w], tH[k][h] (one entry per row: broadcast reads)
// (QM false: d-major, tD[k][d] -- the many-spike kernels, whose 4 reads per quad then share one
// address register)
template <bool QM>
__device__ __forceinline__ void point_tables(const int* act, int na, int H, int W, int D, int NQ, float sgn,
                                             float2* tD, float2* tW, float2* tH) {
  for (int t = threadIdx.x; t < na * 4 * NQ; t += POINT_NT) {
    const int k = t / (4 * NQ), r = t - k * 4 * NQ;
    const int d = QM ? 4 * (r % NQ) + r / NQ : r;
    tD[t] = d < D ? cis_f(mulmod(act[3 + 4 * k], d, D), D, sgn) : make_float2(0.f, 0.f);
  }
  for (int t = threadIdx.x; t < na * W; t += POINT_NT) {
    const int k = t / W, w = t - k * W;
    tW[t] = cis_f(mulmod(act[2 + 4 * k], w, W), W, sgn);
  }
  for (int t = threadIdx.x; t < na * H; t += POINT_NT) {
    const int k = t / H, h = t - k * H;
    tH[t] = cis_f(mulmod(act[1 + 4 * k], h, H), H, sgn);
  }
}

// A thread's rounds: QU quads POINT_NT apart per round, consecutive rounds STEP quads apart.  The
// (h, w, quad) of each slot is advanced by STEP with two carries instead of divided out per quad, and
// the row offset is 32-bit (point_strides_ok); a used quad travels as one code h << 20 | w << 10 | q
// (-1 past the range: its values are 0).
template <int QU>
struct QuadWalk {
  static constexpr int STEP = QU * POINT_NT;
  typedef float Vals[QU][4];
  typedef int Codes[QU];
  const float* xb;
  uint32_t xsh, xsw;
  int qb, qe, nq, W, D;
  int dq, dw, dh;  // STEP = (dh W + dw) nq + dq
  struct State {
    int lin[QU], h[QU], w[QU], q[QU];
  };
  __device__ __forceinline__ static QuadWalk make(const float* xb, int64_t xsh, int64_t xsw, int qb, int qe, int nq,
                                                  int W, int D) {
    QuadWalk k{xb, (uint32_t)xsh, (uint32_t)xsw, qb, qe, nq, W, D, 0, 0, 0};
    const int rows = STEP / nq;
    k.dq = STEP - rows * nq;
    k.dh = rows / W;
    k.dw = rows - k.dh * W;
    return k;
  }
  __device__ __forceinline__ void init(int q0, State& s) const {
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      const int l = q0 + u * POINT_NT, t = l < qe ? l : qb;
      const int h = t / (W * nq), r = t - h * (W * nq), w = r / nq;
      s.lin[u] = l;
      s.h[u] = h;
      s.w[u] = w;
      s.q[u] = r - w * nq;
    }
  }
  __device__ __forceinline__ void load(State& s, Vals& v, Codes& c) const {
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      const bool ok = s.lin[u] < qe;
      const uint32_t off = ok ? (uint32_t)s.h[u] * xsh + (uint32_t)s.w[u] * xsw : 0u;
      load_quad(xb + off, 4 * s.q[u], D, ok && 4 * s.q[u] < D, v[u]);
      c[u] = ok ? (s.h[u] << 20) | (s.w[u] << 10) | s.q[u] : -1;
      // next round
      s.lin[u] += STEP;
      int q = s.q[u] + dq, w = s.w[u] + dw, h = s.h[u] + dh;
      const bool cq = q >= nq;
      q -= cq ? nq : 0;
      w += cq ? 1 : 0;
      const bool cw = w >= W;
      w -= cw ? W : 0;
      h += cw ? 1 : 0;
      s.q[u] = q;
      s.w[u] = w;
      s.h[u] = h;
    }
  }
  // body(values, codes) over every round of [qb, qe) from thread tid with the next DEPTH - 1 rounds'
  // loads in flight while the current one is used (DEPTH 1: load, use, load, ... -- the many-spike
  // kernels, whose bodies need the registers)
  template <int DEPTH, class F>
  __device__ __forceinline__ void run(int tid, F&& body) const {
    State s;
    init(qb + tid, s);
    Vals va, vb, vc;
    Codes ca, cb, cc;
    if (DEPTH == 1) {
      while (s.lin[0] < qe) {
        load(s, va, ca);
        body(va, ca);
      }
    } else if (DEPTH == 2) {
      load(s, va, ca);
      while (ca[0] >= 0) {
        load(s, vb, cb);
        body(va, ca);
        if (cb[0] < 0) break;
        load(s, va, ca);
        body(vb, cb);
      }
    } else {
      load(s, va, ca);
      load(s, vb, cb);
      while (true) {
        if (ca[0] < 0) break;
        load(s, vc, cc);
        body(va, ca);
        if (cb[0] < 0) break;
        load(s, va, ca);
        body(vb, cb);
        if (cc[0] < 0) break;
        load(s, vb, cb);
        body(vc, cc);
      }
    }
  }
};

__device__ __forceinline__ void quad_decode(int code, int& h, int& w, int& q) {
  h = code >> 20;
  w = (code >> 10) & 1023;
  q = code & 1023;
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <int NA>  // most spikes per volume-channel the launch handles (1, or TB_MAX_OPS)
__global__ __launch_bounds__(POINT_NT) void k_point_dft(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int part = (int)blockIdx.x, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ int act[PT_ACT];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  if (na == 0) return;
  const int NQ = (D + 3) / 4, TQ = 4 * NQ;
  // the D factors again as float64 pairs (exact widenings of the float table: the inner product's
  // FMAs then read them without two conversions per voxel and spike)
  double2* tDd = reinterpret_cast<double2*>(smem);
  float2* tD = reinterpret_cast<float2*>(tDd + a.namax * TQ);  // e^{-2 pi i f . n / N}, per axis
  float2* tW = tD + a.namax * TQ;
  float2* tH = tW + a.namax * W;
  double* red = reinterpret_cast<double*>(tH + a.namax * H);  // [4 waves][TB_MAX_OPS][2]
  point_tables<NA == 1>(act, na, H, W, D, NQ, -1.f, tD, tW, tH);
  __syncthreads();
  for (int t = tid; t < na * TQ; t += POINT_NT) tDd[t] = make_double2((double)tD[t].x, (double)tD[t].y);
  __syncthreads();
  const int nrow = W * NQ;
  const int64_t nall = (int64_t)H * nrow;
  // one spike: two rounds (8 KB per wave) in flight -- the read-only stream has nothing else to cover
  // the HBM latency with
  constexpr int QU = PT_QU;
  using QW = QuadWalk<QU>;
  const QW qw = QW::make(a.x + (int64_t)bc * a.xsbc, a.xsh, a.xsw, (int)(nall * part / a.parts),
                         (int)(nall * (part + 1) / a.parts), NQ, W, D);
  // float64 sums: the coefficient of a bin whose value is cancellation noise (the DC of a zero-mean
  // channel) keeps the sign of the exact sum, as the reference's FFT mostly does
  double accr[NA], acci[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) accr[k] = acci[k] = 0.0;
  qw.template run<NA == 1 ? 3 : 1>(tid, [&](const typename QW::Vals& v, const typename QW::Codes& cd) {
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      if (NA > 1 && cd[u] < 0) break;
      int h, w, q;
      quad_decode(cd[u] < 0 ? 0 : cd[u], h, w, q);  // past the range: the values are 0, any twiddles do
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        if (k >= na) break;
        const double2* t = tDd + 4 * k * NQ + (NA == 1 ? q : 4 * q);
        double sr = 0.0, si = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double2 tj = t[NA == 1 ? j * NQ : j];
          sr = fma((double)v[u][j], tj.x, sr);
          si = fma((double)v[u][j], tj.y, si);
        }
        const float2 rr = cmul(tW[k * W + w], tH[k * H + h]);
        accr[k] += sr * (double)rr.x - si * (double)rr.y;
        acci[k] += sr * (double)rr.y + si * (double)rr.x;
      }
    }
  });
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    if (k >= na) break;
    const double vr = wave_sum(accr[k]), vi = wave_sum(acci[k]);
    if (lane == 0) {
      red[(wv * TB_MAX_OPS + k) * 2] = vr;
      red[(wv * TB_MAX_OPS + k) * 2 + 1] = vi;
    }
  }
  __syncthreads();
  if (tid < na) {
    const int k = tid;
    double vr = 0.0, vi = 0.0;
    for (int w = 0; w < POINT_NT / 64; ++w) {
      vr += red[(w * TB_MAX_OPS + k) * 2];
      vi += red[(w * TB_MAX_OPS + k) * 2 + 1];
    }
    double* o = a.part + ((int64_t)(bcl * a.parts + part) * TB_MAX_OPS + act[4 + 4 * k]) * 2;
    o[0] = vr;
    o[1] = vi;
  }
}

__global__ __launch_bounds__(64) void k_point_delta(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  const int bcl = (int)blockIdx.x, lane = (int)threadIdx.x;
  const int s = bcl / a.C, c = bcl - s * a.C;
  const tb_sample_ops& so = a.ops.s[s];
  const double invN = 1.0 / ((double)a.H * (double)a.W * (double)a.D);
  if (bcl == 0 && lane == 0) *a.cnt = 0u;  // k_point_apply's arrival counter
  for (int o = 0; o < TB_MAX_OPS; ++o) {
    const bool on = o < so.n && !(so.op[o].chan >= 0 && so.op[o].chan != c);
    float2 dl = make_float2(0.f, 0.f);
    if (on) {
      double kr = 0.0, ki = 0.0;
      for (int i = lane; i < a.parts; i += 64) {
        const double* p = a.part + ((int64_t)(bcl * a.parts + i) * TB_MAX_OPS + o) * 2;
        kr += p[0];
        ki += p[1];
      }
      kr = wave_sum(kr);
      ki = wave_sum(ki);
      // target value (fft_core.h spike_target, in float64): |K| := amp, phase kept or overridden
      const tb_op& op = so.op[o];
      const double amp = (double)op.f[0];
      double tr, ti;
      if (op.f[1] != op.f[1]) {
        const double m = sqrt(kr * kr + ki * ki);
        tr = m > 0.0 ? amp * kr / m : amp;
        ti = m > 0.0 ? amp * ki / m : 0.0;
      } else {
        tr = amp * (double)op.f[2];
        ti = amp * (double)op.f[3];
      }
      dl = make_float2((float)((tr - kr) * invN), (float)((ti - ki) * invN));
    }
    if (lane == 0) reinterpret_cast<float2*>(a.delta)[bcl * TB_MAX_OPS + o] = dl;
  }
}

template <int NA>
__global__ __launch_bounds__(POINT_NT) void k_point_apply(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int part = (int)blockIdx.x, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x;
  __shared__ int act[PT_ACT];
  __shared__ float2 dls[TB_MAX_OPS];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  const int ncol = D + a.ypad;
  const int NQ = (ncol + 3) / 4, TQ = 4 * NQ;  // quads of output columns (the table is zero past D)
  float2* tD = reinterpret_cast<float2*>(smem);  // e^{+2 pi i f . n / N} factors, per axis
  float2* tW = tD + a.namax * TQ;
  float2* tH = tW + a.namax * W;
  float* red = reinterpret_cast<float*>(tH + a.namax * H);
  point_tables<NA == 1>(act, na, H, W, D, NQ, 1.f, tD, tW, tH);
  if (tid < na) dls[tid] = reinterpret_cast<const float2*>(a.delta)[bcl * TB_MAX_OPS + act[4 + 4 * tid]];
  __syncthreads();
  float* yb = a.y + (int64_t)bc * a.ysbc;
  const bool vout = (a.ysw & 3) == 0 && (a.ysh & 3) == 0 && (reinterpret_cast<uintptr_t>(yb) & 15) == 0;
  const bool vfull = vout && (ncol & 3) == 0;
  const int nrow = W * NQ;
  const int64_t nall = (int64_t)H * nrow;
  using QW = QuadWalk<PT_QU>;
  const QW qw = QW::make(a.x + (int64_t)bc * a.xsbc, a.xsh, a.xsw, (int)(nall * part / a.parts_apply),
                         (int)(nall * (part + 1) / a.parts_apply), NQ, W, D);
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  qw.template run<NA == 1 ? 2 : 1>(tid, [&](const typename QW::Vals& vin, const typename QW::Codes& cd) {
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      if (cd[u] < 0) break;
      int h, w, q;
      quad_decode(cd[u], h, w, q);
      const int d0 = 4 * q;
      float v[4] = {vin[u][0], vin[u][1], vin[u][2], vin[u][3]};
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        if (k >= na) break;
        const float2 rr = cmul(dls[k], cmul(tH[k * H + h], tW[k * W + w]));
        const float2* t = tD + 4 * k * NQ + (NA == 1 ? q : 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 tj = t[NA == 1 ? j * NQ : j];  // zero past D: the padding stays 0
          v[j] += rr.x * tj.x - rr.y * tj.y;
        }
      }
      float vl[4], vh[4];  // columns past D (the zero padding) left out of the min / max
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vl[j] = d0 + j < D ? v[j] : 3.402823466e38f;
        vh[j] = d0 + j < D ? v[j] : -3.402823466e38f;
      }
      lo = min3_raw(min3_raw(lo, vl[0], vl[1]), vl[2], vl[3]);
      hi = max3_raw(max3_raw(hi, vh[0], vh[1]), vh[2], vh[3]);
      float* yr = yb + ((uint32_t)h * (uint32_t)a.ysh + (uint32_t)w * (uint32_t)a.ysw);
      if (vfull) {  // wave-uniform: every quad of the stored row is whole
        st_stream<TB_NT_STORES>(reinterpret_cast<tb_f4v*>(yr + d0), tb_f4v{v[0], v[1], v[2], v[3]});
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < ncol) yr[d0 + j] = v[j];
      }
    }
  });
  if (!a.mm) return;
  // per-workgroup (min, max), then the last workgroup to arrive writes every sample's keys (no
  // same-address atomics from thousands of workgroups)
  lo = wave_min(lo);
  hi = wave_max(hi);
  const int lane = tid & 63, wid = tid >> 6;
  if (lane == 0) {
    red[wid] = lo;
    red[4 + wid] = hi;
  }
  __syncthreads();
  __shared__ int last;
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) {
      lo = fminf(lo, red[w]);
      hi = fmaxf(hi, red[4 + w]);
    }
    store_partial(a.mmp + bcl * a.parts_apply + part, make_float2(lo, hi));
    last = arrive_last(a.cnt, gridDim.x * gridDim.y);
  }
  __syncthreads();
  if (!last) return;
  const int nb = a.nbc / a.C, per = a.C * a.parts_apply;
  for (int b = 0; b < nb; ++b) {
    const float2* p = a.mmp + (int64_t)b * per;
    float l2 = 3.402823466e38f, h2 = -3.402823466e38f;
    for (int i0 = tid; i0 < per; i0 += 4 * POINT_NT) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i0 + u * POINT_NT < per ? load_partial(p + i0 + u * POINT_NT) : make_float2(l2, h2);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        l2 = fminf(l2, v[u].x);
        h2 = fmaxf(h2, v[u].y);
      }
    }
    l2 = wave_min(l2);
    h2 = wave_max(h2);
    __syncthreads();
    if (lane == 0) {
      red[wid] = l2;
      red[4 + wid] = h2;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < 4; ++w) {
        l2 = fminf(l2, red[w]);
        h2 = fmaxf(h2, red[4 + w]);
      }
      const int sb = a.bc0 / a.C + b;
      a.mm[2 * sb] = f2key(l2);
      a.mm[2 * sb + 1] = f2key(h2);
    }
  }
}

bool point_program(const tb_sample_ops& s, int H, int W, int D) {
  if (s.n < 1 || D < 4 || (size_t)TB_MAX_OPS * (H + W + D + 3) * sizeof(float2) > 65536) return false;
  // k_point_dft adds the float64 D table (and its wave sums)
  if ((size_t)TB_MAX_OPS * ((H + W + D + 3) * sizeof(float2) + (D + 3) * sizeof(double2)) +
          4 * TB_MAX_OPS * 2 * sizeof(double) > 163840)
    return false;
  for (int o = 0; o < s.n; ++o)
    if (s.op[o].kind != TB_OP_SPIKE) return false;
  const int n[3] = {H, W, D};
  for (int o = 0; o < s.n; ++o)
    for (int q = 0; q < o; ++q) {
      const tb_op &A = s.op[o], &B = s.op[q];
      if (A.chan >= 0 && B.chan >= 0 && A.chan != B.chan) continue;
      bool same = true, conj = true;
      for (int ax = 0; ax < 3; ++ax) {
        same &= A.i[ax] == B.i[ax];
        conj &= A.i[ax] == (n[ax] - B.i[ax]) % n[ax];
      }
      if (same || conj) return false;
    }
  return true;
}

static size_t point_lds(const PointArgs& a, int stage) {
  const int tq = stage == 0 ? 4 * ((a.D + 3) / 4) : 4 * ((a.D + a.ypad + 3) / 4);
  const size_t tabs = (size_t)a.namax * (tq + a.W + a.H) * sizeof(float2);
  return stage == 0 ? (size_t)a.namax * tq * sizeof(double2) + tabs + 4 * TB_MAX_OPS * 2 * sizeof(double)
                    : tabs + 2 * POINT_NT / 64 * sizeof(float);
}

typedef void (*PointKern)(PointArgs);

static PointKern point_dft_kernel(const PointArgs& a) {
  return a.namax == 1 ? k_point_dft<1> : k_point_dft<TB_MAX_OPS>;
}

template <class K>
static int point_parts(K kern, size_t lds, int nbc, int ncu) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  int occ = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(reinterpret_cast<const void*>(kern), lds);
    auto it = cache.find(key);
    if (it != cache.end()) {
      occ = it->second;
    } else {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, POINT_NT, lds) != hipSuccess || occ < 1) occ = 4;
      cache[key] = occ;
    }
  }
  int g = ncu * occ;
  g = g > POINT_WG ? POINT_WG : g;
  const int parts = g / nbc;
  return parts < 1 ? 1 : parts;
}

void point_grid(PointArgs& a, int ncu) {
  // occupancy is queried at the launch's LDS size
  const PointKern kd = point_dft_kernel(a);
  const auto ka = a.namax == 1 ? k_point_apply<1> : k_point_apply<TB_MAX_OPS>;
  (void)allow_lds(kd, point_lds(a, 0));
  a.parts = point_parts(kd, point_lds(a, 0), a.nbc, ncu);
  (void)allow_lds(ka, point_lds(a, 2));
  a.parts_apply = point_parts(ka, point_lds(a, 2), a.nbc, ncu);
}

hipError_t launch_point(const PointArgs& a, hipStream_t st, int stage) {
  if (stage == 0) {
    const PointKern kd = point_dft_kernel(a);
    const hipError_t e = allow_lds(kd, point_lds(a, 0));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kd, dim3(a.parts, a.nbc), dim3(POINT_NT), point_lds(a, 0), st, a);
  } else if (stage == 1) {
    hipLaunchKernelGGL(k_point_delta, dim3(a.nbc), dim3(64), 0, st, a);
  } else {
    const auto ka = a.namax == 1 ? k_point_apply<1> : k_point_apply<TB_MAX_OPS>;
    const hipError_t e = allow_lds(ka, point_lds(a, 2));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ka, dim3(a.parts_apply, a.nbc), dim3(POINT_NT), point_lds(a, 2), st, a);
  }
  return hipGetLastError();
}

}  // namespace tb
