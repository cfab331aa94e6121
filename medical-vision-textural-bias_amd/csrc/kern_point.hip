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

constexpr int PT_RB = 4;  // rows a wave keeps in flight

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

__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float x, float y) { return x + y; });
}

}  // namespace

__global__ __launch_bounds__(POINT_NT) void k_point_dft(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int h = (int)blockIdx.x, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ int act[PT_ACT];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  if (na == 0) return;
  float2* tD = reinterpret_cast<float2*>(smem);       // [na][D]  e^{-2 pi i kd d / D}
  float2* tW = tD + TB_MAX_OPS * D;                    // [na][W]  e^{-2 pi i kw w / W}
  double* red = reinterpret_cast<double*>(tW + TB_MAX_OPS * W);  // [4 waves][na][2]
  for (int t = tid; t < na * D; t += POINT_NT) {
    const int k = t / D, d = t - k * D;
    tD[k * D + d] = cis_f(mulmod(act[3 + 4 * k], d, D), D, -1.f);
  }
  for (int t = tid; t < na * W; t += POINT_NT) {
    const int k = t / W, w = t - k * W;
    tW[k * W + w] = cis_f(mulmod(act[2 + 4 * k], w, W), W, -1.f);
  }
  __syncthreads();
  const float* xs = a.x + (int64_t)bc * a.xsbc + (int64_t)h * a.xsh;
  float accr[TB_MAX_OPS], acci[TB_MAX_OPS];
#pragma unroll
  for (int k = 0; k < TB_MAX_OPS; ++k) accr[k] = acci[k] = 0.f;
  for (int w0 = wv * PT_RB; w0 < W; w0 += 4 * PT_RB) {
    float sr[PT_RB][TB_MAX_OPS], si[PT_RB][TB_MAX_OPS];
#pragma unroll
    for (int r = 0; r < PT_RB; ++r)
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) sr[r][k] = si[r][k] = 0.f;
    for (int d = lane; d < D; d += 64) {
      float xv[PT_RB];
#pragma unroll
      for (int r = 0; r < PT_RB; ++r) xv[r] = w0 + r < W ? xs[(int64_t)(w0 + r) * a.xsw + d] : 0.f;
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) {
        if (k >= na) break;
        const float2 t = tD[k * D + d];
#pragma unroll
        for (int r = 0; r < PT_RB; ++r) {
          sr[r][k] = fmaf(xv[r], t.x, sr[r][k]);
          si[r][k] = fmaf(xv[r], t.y, si[r][k]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < PT_RB; ++r) {
      if (w0 + r >= W) break;
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) {
        if (k >= na) break;
        const float2 t = tW[k * W + w0 + r];
        accr[k] += sr[r][k] * t.x - si[r][k] * t.y;
        acci[k] += sr[r][k] * t.y + si[r][k] * t.x;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < TB_MAX_OPS; ++k) {
    if (k >= na) break;
    const float vr = wave_sum(accr[k]), vi = wave_sum(acci[k]);
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
    double* o = a.part + ((int64_t)(bcl * H + h) * TB_MAX_OPS + act[4 + 4 * k]) * 2;
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
      for (int h = lane; h < a.H; h += 64) {
        const double* p = a.part + ((int64_t)(bcl * a.H + h) * TB_MAX_OPS + o) * 2;
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
  const int h = (int)blockIdx.x, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ int act[PT_ACT];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  float2* tD = reinterpret_cast<float2*>(smem);   // [na][D]  e^{+2 pi i kd d / D}
  float2* R = tD + TB_MAX_OPS * D;                 // [na][W]  Delta / N e^{2 pi i (kh h / H + kw w / W)}
  float* red = reinterpret_cast<float*>(R + TB_MAX_OPS * W);
  for (int t = tid; t < na * D; t += POINT_NT) {
    const int k = t / D, d = t - k * D;
    tD[k * D + d] = cis_f(mulmod(act[3 + 4 * k], d, D), D, 1.f);
  }
  for (int t = tid; t < na * W; t += POINT_NT) {
    const int k = t / W, w = t - k * W;
    const float2 dl = reinterpret_cast<const float2*>(a.delta)[bcl * TB_MAX_OPS + act[4 + 4 * k]];
    // phase (kh h / H + kw w / W) as one exact fraction of H W, reduced once
    const int64_t num = ((int64_t)mulmod(act[1 + 4 * k], h, H) * W + (int64_t)mulmod(act[2 + 4 * k], w, W) * H) %
                        ((int64_t)H * W);
    double s, c;
    sincospi(2.0 * (double)num / ((double)H * (double)W), &s, &c);
    R[k * W + w] = make_float2((float)(dl.x * c - dl.y * s), (float)(dl.x * s + dl.y * c));
  }
  __syncthreads();
  const float* xs = a.x + (int64_t)bc * a.xsbc + (int64_t)h * a.xsh;
  float* ys = a.y + (int64_t)bc * a.ysbc + (int64_t)h * a.ysh;
  const int ncol = D + a.ypad;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int w0 = wv * PT_RB; w0 < W; w0 += 4 * PT_RB) {
    for (int d = lane; d < ncol; d += 64) {
      float v[PT_RB];
      const bool img = d < D;
#pragma unroll
      for (int r = 0; r < PT_RB; ++r) v[r] = (img && w0 + r < W) ? xs[(int64_t)(w0 + r) * a.xsw + d] : 0.f;
      if (img) {
#pragma unroll
        for (int k = 0; k < TB_MAX_OPS; ++k) {
          if (k >= na) break;
          const float2 t = tD[k * D + d];
#pragma unroll
          for (int r = 0; r < PT_RB; ++r) {
            if (w0 + r < W) {
              const float2 q = R[k * W + w0 + r];
              v[r] += q.x * t.x - q.y * t.y;
            }
          }
        }
#pragma unroll
        for (int r = 0; r < PT_RB; ++r)
          if (w0 + r < W) {
            lo = fminf(lo, v[r]);
            hi = fmaxf(hi, v[r]);
          }
      }
#pragma unroll
      for (int r = 0; r < PT_RB; ++r)
        if (w0 + r < W) ys[(int64_t)(w0 + r) * a.ysw + d] = v[r];
    }
  }
  if (a.mm) block_minmax_atomic<POINT_NT>(lo, hi, red, a.mm + 2 * (bc / a.C));
}

bool point_program(const tb_sample_ops& s, int H, int W, int D) {
  if (s.n < 1 || (size_t)TB_MAX_OPS * (W + D) * sizeof(float2) > 65536) return false;
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
  return (size_t)bc * H * TB_MAX_OPS * 2 * sizeof(double) + (size_t)bc * TB_MAX_OPS * 2 * sizeof(float) + 256;
}

hipError_t launch_point(const PointArgs& a, hipStream_t st, int stage) {
  const size_t tabs = (size_t)TB_MAX_OPS * (a.D + a.W) * sizeof(float2);
  if (stage == 0) {
    hipLaunchKernelGGL(k_point_dft, dim3(a.H, a.nbc), dim3(POINT_NT), tabs + 4 * TB_MAX_OPS * 2 * sizeof(double), st, a);
  } else if (stage == 1) {
    hipLaunchKernelGGL(k_point_delta, dim3(a.nbc), dim3(64), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_point_apply, dim3(a.H, a.nbc), dim3(POINT_NT), tabs + 2 * POINT_NT / 64 * sizeof(float), st, a);
  }
  return hipGetLastError();
}

}  // namespace tb
