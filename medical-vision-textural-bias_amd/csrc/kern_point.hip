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

__device__ __forceinline__ void load_quad(const float* row, int d0, int D, bool vec, float (&v)[4]) {
  if (vec && d0 + 4 <= D) {
    const float4 q = *reinterpret_cast<const float4*>(row + d0);
    v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = d0 + j < D ? row[d0 + j] : 0.f;
  }
}

// per-axis twiddle tables of the active spikes: t[k][i] = e^{sgn 2 pi i f_k,axis i / n}, i < n (+3 zero
// entries past D for the partial last quad)
__device__ __forceinline__ void point_tables(const int* act, int na, int H, int W, int D, float sgn, float2* tD,
                                             float2* tW, float2* tH) {
  const int Dp = D + 3;
  for (int t = threadIdx.x; t < na * Dp; t += POINT_NT) {
    const int k = t / Dp, d = t - k * Dp;
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

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

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
  const int Dp = D + 3;
  // the D factors again as float64 pairs (exact widenings of the float table: the inner product's
  // FMAs then read them without two conversions per voxel and spike)
  double2* tDd = reinterpret_cast<double2*>(smem);
  float2* tD = reinterpret_cast<float2*>(tDd + a.namax * Dp);  // e^{-2 pi i f . n / N}, [namax][n] per axis
  float2* tW = tD + a.namax * Dp;
  float2* tH = tW + a.namax * W;
  double* red = reinterpret_cast<double*>(tH + a.namax * H);  // [4 waves][TB_MAX_OPS][2]
  point_tables(act, na, H, W, D, -1.f, tD, tW, tH);
  __syncthreads();
  for (int t = tid; t < na * Dp; t += POINT_NT) tDd[t] = make_double2((double)tD[t].x, (double)tD[t].y);
  __syncthreads();
  const float* xb = a.x + (int64_t)bc * a.xsbc;
  const bool vec = (a.xsw & 3) == 0 && (a.xsh & 3) == 0 && (reinterpret_cast<uintptr_t>(xb) & 15) == 0;
  const int nq = (D + 3) / 4, nrow = W * nq;
  const int64_t nall = (int64_t)H * nrow;
  const int qb = (int)(nall * part / a.parts), qe = (int)(nall * (part + 1) / a.parts);
  const FastDiv frow = FastDiv::make(nrow), fq = FastDiv::make(nq);
  // float64 sums: the coefficient of a bin whose value is cancellation noise (the DC of a zero-mean
  // channel) keeps the sign of the exact sum, as the reference's FFT mostly does
  double accr[TB_MAX_OPS], acci[TB_MAX_OPS];
#pragma unroll
  for (int k = 0; k < TB_MAX_OPS; ++k) accr[k] = acci[k] = 0.0;
  for (int q0 = qb + tid; q0 < qe; q0 += PT_QU * POINT_NT) {
    float v[PT_QU][4];
    int hh[PT_QU], ww[PT_QU], dd[PT_QU];
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      const int q = q0 + u * POINT_NT < qe ? q0 + u * POINT_NT : qb;
      const int h = frow.div(q), r = q - h * nrow, w = fq.div(r);
      hh[u] = q0 + u * POINT_NT < qe ? h : -1;
      ww[u] = w;
      dd[u] = 4 * (r - w * nq);
      load_quad(xb + (int64_t)h * a.xsh + (int64_t)w * a.xsw, dd[u], hh[u] >= 0 ? D : 0, vec, v[u]);
    }
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      if (hh[u] < 0) break;
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) {
        if (k >= na) break;
        const double2* t = tDd + k * Dp + dd[u];
        double sr = 0.0, si = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double2 tj = t[j];
          sr = fma((double)v[u][j], tj.x, sr);
          si = fma((double)v[u][j], tj.y, si);
        }
        const float2 r = cmul(tW[k * W + ww[u]], tH[k * H + hh[u]]);
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

__global__ __launch_bounds__(POINT_NT) void k_point_apply(PointArgs) {
  const PointArgs& a = kargs<PointArgs>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int part = (int)blockIdx.x, bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int H = a.H, W = a.W, D = a.D, tid = (int)threadIdx.x;
  __shared__ int act[PT_ACT];
  __shared__ float2 dls[TB_MAX_OPS];
  point_active(a, bcl, act);
  const int na = __builtin_amdgcn_readfirstlane(act[0]);
  const int Dp = D + 3;
  float2* tD = reinterpret_cast<float2*>(smem);  // e^{+2 pi i f . n / N} factors, [namax][n] per axis
  float2* tW = tD + a.namax * Dp;
  float2* tH = tW + a.namax * W;
  float* red = reinterpret_cast<float*>(tH + a.namax * H);
  point_tables(act, na, H, W, D, 1.f, tD, tW, tH);
  if (tid < na) dls[tid] = reinterpret_cast<const float2*>(a.delta)[bcl * TB_MAX_OPS + act[4 + 4 * tid]];
  __syncthreads();
  const float* xb = a.x + (int64_t)bc * a.xsbc;
  float* yb = a.y + (int64_t)bc * a.ysbc;
  const int ncol = D + a.ypad;
  const bool vin = (a.xsw & 3) == 0 && (a.xsh & 3) == 0 && (reinterpret_cast<uintptr_t>(xb) & 15) == 0;
  const bool vout = (a.ysw & 3) == 0 && (a.ysh & 3) == 0 && (reinterpret_cast<uintptr_t>(yb) & 15) == 0;
  const int nq = (ncol + 3) / 4, nrow = W * nq;  // quads of output columns
  const int64_t nall = (int64_t)H * nrow;
  const int qb = (int)(nall * part / a.parts_apply), qe = (int)(nall * (part + 1) / a.parts_apply);
  const FastDiv frow = FastDiv::make(nrow), fq = FastDiv::make(nq);
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int q0 = qb + tid; q0 < qe; q0 += PT_QU * POINT_NT) {
    float v[PT_QU][4];
    int hh[PT_QU], ww[PT_QU], dd[PT_QU];
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      const int q = q0 + u * POINT_NT < qe ? q0 + u * POINT_NT : qb;
      const int h = frow.div(q), r = q - h * nrow, w = fq.div(r);
      hh[u] = q0 + u * POINT_NT < qe ? h : -1;
      ww[u] = w;
      dd[u] = 4 * (r - w * nq);
      load_quad(xb + (int64_t)h * a.xsh + (int64_t)w * a.xsw, dd[u], hh[u] >= 0 ? D : 0, vin, v[u]);
    }
#pragma unroll
    for (int u = 0; u < PT_QU; ++u) {
      if (hh[u] < 0) break;
      const int d0 = dd[u];
#pragma unroll
      for (int k = 0; k < TB_MAX_OPS; ++k) {
        if (k >= na) break;
        const float2 r = cmul(dls[k], cmul(tH[k * H + hh[u]], tW[k * W + ww[u]]));
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
      float* yr = yb + (int64_t)hh[u] * a.ysh + (int64_t)ww[u] * a.ysw;
      if (vout && d0 + 4 <= ncol) {
        *reinterpret_cast<float4*>(yr + d0) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < ncol) yr[d0 + j] = v[u][j];
      }
    }
  }
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
  if (s.n < 1 || (size_t)TB_MAX_OPS * (H + W + D + 3) * sizeof(float2) > 65536) return false;
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
  const size_t tabs = (size_t)a.namax * (a.D + 3 + a.W + a.H) * sizeof(float2);
  return stage == 0 ? (size_t)a.namax * (a.D + 3) * sizeof(double2) + tabs + 4 * TB_MAX_OPS * 2 * sizeof(double)
                    : tabs + 2 * POINT_NT / 64 * sizeof(float);
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
  (void)allow_lds(k_point_dft, point_lds(a, 0));  // occupancy is queried at the launch's LDS size
  a.parts = point_parts(k_point_dft, point_lds(a, 0), a.nbc, ncu);
  a.parts_apply = point_parts(k_point_apply, point_lds(a, 2), a.nbc, ncu);
}

hipError_t launch_point(const PointArgs& a, hipStream_t st, int stage) {
  if (stage == 0) {
    const hipError_t e = allow_lds(k_point_dft, point_lds(a, 0));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_point_dft, dim3(a.parts, a.nbc), dim3(POINT_NT), point_lds(a, 0), st, a);
  } else if (stage == 1) {
    hipLaunchKernelGGL(k_point_delta, dim3(a.nbc), dim3(64), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_point_apply, dim3(a.parts_apply, a.nbc), dim3(POINT_NT), point_lds(a, 2), st, a);
  }
  return hipGetLastError();
}

}  // namespace tb
