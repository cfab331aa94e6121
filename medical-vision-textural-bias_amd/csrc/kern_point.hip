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

// Work item = a quad: 4 consecutive columns d0 .. d0 + 3 of one row w of the slab; consecutive lanes
// take consecutive quads (coalesced), each thread PT_QU quads per round with all their loads issued
// first (a wave per row kept ~4 loads in flight: 230 us at C3 against ~40 for the bytes).
constexpr int PT_QU = 4;
// Workgroups per slab: each takes a quarter of the slab's quads, so a C3 launch is 7,680 small
// workgroups rather than 1,920 slabs (one full round of resident workgroups plus a 7 % second round
// took twice one round's time).
constexpr int PT_PARTS = 4;

__device__ __forceinline__ void load_quad(const float* row, int d0, int D, bool vec, float (&v)[4]) {
  if (vec && d0 + 4 <= D) {
    const float4 q = *reinterpret_cast<const float4*>(row + d0);
    v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = d0 + j < D ? row[d0 + j] : 0.f;
  }
}

__global__ __launch_bounds__(POINT_NT) void k_point_dft(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int h = (int)blockIdx.x / PT_PARTS, part = (int)blockIdx.x - h * PT_PARTS, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ int act[PT_ACT];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  if (na == 0) return;
  float2* tD = reinterpret_cast<float2*>(smem);       // [na][D + 3]  e^{-2 pi i kd d / D}, 0 past D
  float2* tW = tD + TB_MAX_OPS * (D + 3);              // [na][W]  e^{-2 pi i kw w / W}
  double* red = reinterpret_cast<double*>(tW + TB_MAX_OPS * W);  // [4 waves][TB_MAX_OPS][2]
  const int Dp = D + 3;
  for (int t = tid; t < na * Dp; t += POINT_NT) {
    const int k = t / Dp, d = t - k * Dp;
    tD[t] = d < D ? cis_f(mulmod(act[3 + 4 * k], d, D), D, -1.f) : make_float2(0.f, 0.f);
  }
  for (int t = tid; t < na * W; t += POINT_NT) {
    const int k = t / W, w = t - k * W;
    tW[t] = cis_f(mulmod(act[2 + 4 * k], w, W), W, -1.f);
  }
  __syncthreads();
  const float* xs = a.x + (int64_t)bc * a.xsbc + (int64_t)h * a.xsh;
  const bool vec = (a.xsw & 3) == 0 && (reinterpret_cast<uintptr_t>(xs) & 15) == 0;
  const int nq = (D + 3) / 4, nall = W * nq;
  const int qb = (int)((int64_t)nall * part / PT_PARTS), nquad = (int)((int64_t)nall * (part + 1) / PT_PARTS);
  const FastDiv fq = FastDiv::make(nq);
  // float64 sums: the coefficient of a bin whose value is cancellation noise (the DC of a zero-mean
  // channel) keeps the sign of the exact sum, as the reference's FFT mostly does
  double accr[TB_MAX_OPS], acci[TB_MAX_OPS];
#pragma unroll
  for (int k = 0; k < TB_MAX_OPS; ++k) accr[k] = acci[k] = 0.0;
  for (int q0 = qb + tid; q0 < nquad; q0 += PT_QU * POINT_NT) {
    float v[PT_QU][4];
    int ww[PT_QU], dd[PT_QU];
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      const int q = q0 + u * POINT_NT;
      const int w = fq.div(q < nquad ? q : qb);
      ww[u] = q < nquad ? w : -1;
      dd[u] = 4 * ((q < nquad ? q : qb) - w * nq);
      load_quad(xs + (int64_t)w * a.xsw, dd[u], q < nquad ? D : 0, vec, v[u]);
    }
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      if (ww[u] < 0) break;
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) {
        if (k >= na) break;
        const float2* t = tD + k * Dp + dd[u];
        double sr = 0.0, si = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 tj = t[j];
          sr = fma((double)v[u][j], (double)tj.x, sr);
          si = fma((double)v[u][j], (double)tj.y, si);
        }
        const float2 r = tW[k * W + ww[u]];
        accr[k] += sr * (double)r.x - si * (double)r.y;
        acci[k] += sr * (double)r.y + si * (double)r.x;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < TB_MAX_OPS; ++k) {
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
    double s, c;
    sincospi(2.0 * (double)mulmod(act[1 + 4 * k], h, H) / (double)H, &s, &c);  // e^{-2 pi i kh h / H}
    double* o = a.part + ((int64_t)(bcl * H * PT_PARTS + blockIdx.x) * TB_MAX_OPS + act[4 + 4 * k]) * 2;
    o[0] = vr * c + vi * s;
    o[1] = vi * c - vr * s;
  }
}

__global__ __launch_bounds__(64) void k_point_delta(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  const int bcl = (int)blockIdx.x, lane = (int)threadIdx.x;
  const int s = bcl / a.C, c = bcl - s * a.C;
  const tb_sample_ops& so = a.ops.s[s];
  const double invN = 1.0 / ((double)a.H * (double)a.W * (double)a.D);
  for (int o = 0; o < TB_MAX_OPS; ++o) {
    const bool on = o < so.n && !(so.op[o].chan >= 0 && so.op[o].chan != c);
    float2 dl = make_float2(0.f, 0.f);
    if (on) {
      double kr = 0.0, ki = 0.0;
      for (int h = lane; h < a.H * PT_PARTS; h += 64) {
        const double* p = a.part + ((int64_t)(bcl * a.H * PT_PARTS + h) * TB_MAX_OPS + o) * 2;
        kr += p[0];
        ki += p[1];
      }
      for (int off = 32; off > 0; off >>= 1) {
        kr += __shfl_xor(kr, off);
        ki += __shfl_xor(ki, off);
      }
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

__global__ __launch_bounds__(POINT_NT) void k_point_apply(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int h = (int)blockIdx.x / PT_PARTS, part = (int)blockIdx.x - h * PT_PARTS, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x;
  __shared__ int act[PT_ACT];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  const int Dp = D + 3;
  float2* tD = reinterpret_cast<float2*>(smem);   // [na][D + 3]  e^{+2 pi i kd d / D}, 0 past D
  float2* R = tD + TB_MAX_OPS * Dp;                // [na][W]  Delta / N e^{2 pi i (kh h / H + kw w / W)}
  float* red = reinterpret_cast<float*>(R + TB_MAX_OPS * W);
  for (int t = tid; t < na * Dp; t += POINT_NT) {
    const int k = t / Dp, d = t - k * Dp;
    tD[t] = d < D ? cis_f(mulmod(act[3 + 4 * k], d, D), D, 1.f) : make_float2(0.f, 0.f);
  }
  for (int t = tid; t < na * W; t += POINT_NT) {
    const int k = t / W, w = t - k * W;
    const float2 dl = reinterpret_cast<const float2*>(a.delta)[bcl * TB_MAX_OPS + act[4 + 4 * k]];
    // phase (kh h / H + kw w / W) as one exact fraction of H W, reduced once
    const int64_t num = ((int64_t)mulmod(act[1 + 4 * k], h, H) * W + (int64_t)mulmod(act[2 + 4 * k], w, W) * H) %
                        ((int64_t)H * W);
    double s, c;
    sincospi(2.0 * (double)num / ((double)H * (double)W), &s, &c);
    R[t] = make_float2((float)(dl.x * c - dl.y * s), (float)(dl.x * s + dl.y * c));
  }
  __syncthreads();
  const float* xs = a.x + (int64_t)bc * a.xsbc + (int64_t)h * a.xsh;
  float* ys = a.y + (int64_t)bc * a.ysbc + (int64_t)h * a.ysh;
  const int ncol = D + a.ypad;
  const bool vin = (a.xsw & 3) == 0 && (reinterpret_cast<uintptr_t>(xs) & 15) == 0;
  const bool vout = (a.ysw & 3) == 0 && (reinterpret_cast<uintptr_t>(ys) & 15) == 0;
  const int nq = (ncol + 3) / 4, nall = W * nq;  // quads of output columns
  const int qb = (int)((int64_t)nall * part / PT_PARTS), nquad = (int)((int64_t)nall * (part + 1) / PT_PARTS);
  const FastDiv fq = FastDiv::make(nq);
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int q0 = qb + tid; q0 < nquad; q0 += PT_QU * POINT_NT) {
    float v[PT_QU][4];
    int ww[PT_QU], dd[PT_QU];
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      const int q = q0 + u * POINT_NT;
      const int w = fq.div(q < nquad ? q : qb);
      ww[u] = q < nquad ? w : -1;
      dd[u] = 4 * ((q < nquad ? q : qb) - w * nq);
      load_quad(xs + (int64_t)w * a.xsw, dd[u], q < nquad ? D : 0, vin, v[u]);
    }
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      if (ww[u] < 0) break;
      const int d0 = dd[u];
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) {
        if (k >= na) break;
        const float2 r = R[k * W + ww[u]];
        const float2* t = tD + k * Dp + (d0 < D ? d0 : 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 tj = t[j];
          v[u][j] += d0 < D ? r.x * tj.x - r.y * tj.y : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (d0 + j < D) {
          lo = fminf(lo, v[u][j]);
          hi = fmaxf(hi, v[u][j]);
        }
      float* yr = ys + (int64_t)ww[u] * a.ysw;
      if (vout && d0 + 4 <= ncol) {
        *reinterpret_cast<float4*>(yr + d0) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < ncol) yr[d0 + j] = v[u][j];
      }
    }
  }
  if (a.mm) block_minmax_atomic<POINT_NT>(lo, hi, red, a.mm + 2 * (bc / a.C));
}

bool point_program(const tb_sample_ops& s, int H, int W, int D) {
  if (s.n < 1 || (size_t)TB_MAX_OPS * (W + D + 3) * sizeof(float2) > 65536) return false;
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

size_t point_workspace_bytes(int H, int bc) {
  return (size_t)bc * H * PT_PARTS * TB_MAX_OPS * 2 * sizeof(double) + (size_t)bc * TB_MAX_OPS * 2 * sizeof(float) + 512;
}

hipError_t launch_point(const PointArgs& a, hipStream_t st, int stage) {
  const size_t tabs = (size_t)TB_MAX_OPS * (a.D + 3 + a.W) * sizeof(float2);
  if (stage == 0) {
    hipLaunchKernelGGL(k_point_dft, dim3(a.H * PT_PARTS, a.nbc), dim3(POINT_NT), tabs + 4 * TB_MAX_OPS * 2 * sizeof(double), st, a);
  } else if (stage == 1) {
    hipLaunchKernelGGL(k_point_delta, dim3(a.nbc), dim3(64), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_point_apply, dim3(a.H * PT_PARTS, a.nbc), dim3(POINT_NT), tabs + 2 * POINT_NT / 64 * sizeof(float), st, a);
  }
  return hipGetLastError();
}

}  // namespace tb
