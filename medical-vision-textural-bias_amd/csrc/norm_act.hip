// norm_act.hip -- fused InstanceNorm3d(affine=False) + PReLU(1 parameter), forward and backward.
//
// The U-Net the reference trains (MONAI UNet, 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199;
// module tree source_code/test.ipynb:754-1010) follows every convolution but the last with an "ADN"
// block: InstanceNorm3d(eps 1e-5, affine=False) -> Dropout(0) -> PReLU(a).  ATen runs that as
// batch_norm over [1, N*C, ...] (few, huge channels: one reduction block per channel) plus separate
// PReLU kernels and a PReLU weight-gradient reduction -- ~30 ms of a 89 ms train step.  Here each
// direction is two HBM sweeps over [N*C instances][S voxels] with the reductions split over the
// whole grid (float64 per-thread partials, then across lanes, blocks and the grid):
//   forward   K1 sums(x) -> K2 y = prelu((x - mean) * rstd)                  read 2S, write S
//   backward  K3 sums(g, g z, dy z [z<=0]) -> K4 dx = rstd (g - mean g - z mean(g z))
//             with z = (x - mean) rstd, g = dy * (z > 0 ? 1 : a)            read 4S, write S
//             (backward arithmetic in float64 per voxel: see K3)
// Statistics: biased variance, rstd = 1/sqrt(var + eps) (torch.nn.functional.instance_norm).
#include <hip/hip_runtime.h>

#include "texbias.h"

namespace {

constexpr int NT = 256;
constexpr int VPT = 16;                    // float4 per thread per chunk
constexpr int CHUNK = NT * VPT * 4;        // voxels per block

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-reduce K doubles and add them atomically to dst[0..K)
template <int K>
__device__ __forceinline__ void block_atomic_add(double (&v)[K], double* dst) {
  __shared__ double red[K][NT / 64];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) red[k][wid] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < K) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[threadIdx.x][w];
    atomicAdd(&dst[threadIdx.x], s);
  }
}

// Visit the chunk of instance `nc` assigned to this block: f(value-index, float4 or scalar lanes).
// S % 4 == 0 (and 16-B aligned base) uses float4 accesses; otherwise scalar.
struct Chunk {
  int64_t base, begin, end;  // element offsets: instance base, [begin, end) within the instance
};
__device__ __forceinline__ Chunk chunk_of(int64_t S) {
  const int64_t nc = blockIdx.y;
  const int64_t b = (int64_t)blockIdx.x * CHUNK;
  const int64_t e = b + CHUNK < S ? b + CHUNK : S;
  return Chunk{nc * S, b, e};
}

__device__ __forceinline__ void stats_of(double s1, double s2, int64_t S, float eps, float& mean, float& rstd) {
  const double m = s1 / (double)S;
  double var = s2 / (double)S - m * m;
  var = var > 0.0 ? var : 0.0;
  mean = (float)m;
  rstd = (float)(1.0 / sqrt(var + (double)eps));
}

__device__ __forceinline__ float prelu(float z, float a) { return z > 0.f ? z : a * z; }

// K1: per-instance sum and sum of squares into acc[nc][2] (zeroed by the caller)
__global__ __launch_bounds__(NT) void k_in_stats(const float* __restrict__ x, double* __restrict__ acc, int64_t S,
                                                 int vec) {
  const Chunk c = chunk_of(S);
  // float64 per thread (x^2 of a float32 is exact in float64): the statistics reach the backward's
  // g - mean g - z mean(g z), whose cancellation at the top of the U-Net turns a 1e-6 error in
  // rstd into a visible one in the input gradient (scripts/diag/grad_noise.py)
  double s1 = 0.0, s2 = 0.0;
  if (vec) {
    const float4* p = reinterpret_cast<const float4*>(x + c.base + c.begin);
    const int n4 = (int)((c.end - c.begin) >> 2);
    float4 v[VPT];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = threadIdx.x + k * NT;
      v[k] = i < n4 ? p[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const double a = v[k].x, b = v[k].y, e = v[k].z, f = v[k].w;
      s1 += (a + b) + (e + f);
      s2 += (a * a + b * b) + (e * e + f * f);
    }
  } else {
    for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) {
      const double v = x[c.base + i];
      s1 += v;
      s2 += v * v;
    }
  }
  double r[2] = {s1, s2};
  block_atomic_add<2>(r, acc + 2 * blockIdx.y);
}

// Channel sums out[c] = sum_{n, s} x[n][c][s] (the bias gradient of a convolution: ATen reduces
// grad_out over (N, D, H, W) with a generic reduction at ~0.1-0.3 TB/s); one HBM sweep, block
// partials in double, one float atomic per block into out (zeroed by the host function).
__global__ __launch_bounds__(NT) void k_channel_sum(const float* __restrict__ x, float* __restrict__ out, int64_t S,
                                                    int C, int vec) {
  const Chunk c = chunk_of(S);
  float s1 = 0.f;
  if (vec) {
    const float4* p = reinterpret_cast<const float4*>(x + c.base + c.begin);
    const int n4 = (int)((c.end - c.begin) >> 2);
    float4 v[VPT];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = threadIdx.x + k * NT;
      v[k] = i < n4 ? p[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) s1 += (v[k].x + v[k].y) + (v[k].z + v[k].w);
  } else {
    for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) s1 += x[c.base + i];
  }
  double r[1] = {(double)s1};
  // block_atomic_add adds doubles; reduce here and add one float
  __shared__ double red[NT / 64];
  r[0] = wave_sum(r[0]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = r[0];
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    atomicAdd(&out[blockIdx.y % C], (float)t);
  }
}

// Dice statistics of the reference's loss (DiceLoss(sigmoid=True, squared_pred=True),
// stylized_gibbs12p5.py:201): per instance nc, acc[nc] += {sum t p, sum t^2 | t, sum p^2 | p} with
// p = sigmoid(x) (flags & 1) -- one fused sweep instead of a sigmoid, two products and three ATen
// reductions of 6 outputs each (~2 ms apiece at 240x240x160).  flags & 2: squared_pred.
__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + expf(-v)); }

__global__ __launch_bounds__(NT) void k_dice_sums(const float* __restrict__ x, const float* __restrict__ t,
                                                  double* __restrict__ acc, int64_t S, int flags, int vec) {
  const Chunk c = chunk_of(S);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  auto add1 = [&](float xv, float tv) {
    float p = (flags & 1) ? sigm(xv) : xv;
    if (flags & 4) p = p >= 0.5f ? 1.f : 0.f;  // the metric's AsDiscrete(threshold 0.5)
    a0 += tv * p;
    if (flags & 2) {
      a1 += tv * tv;
      a2 += p * p;
    } else {
      a1 += tv;
      a2 += p;
    }
  };
  if (vec) {
    const float4* px = reinterpret_cast<const float4*>(x + c.base + c.begin);
    const float4* pt = reinterpret_cast<const float4*>(t + c.base + c.begin);
    const int n4 = (int)((c.end - c.begin) >> 2);
#pragma unroll 4
    for (int k = 0; k < VPT; ++k) {
      const int i = threadIdx.x + k * NT;
      if (i < n4) {
        const float4 xv = px[i], tv = pt[i];
        add1(xv.x, tv.x);
        add1(xv.y, tv.y);
        add1(xv.z, tv.z);
        add1(xv.w, tv.w);
      }
    }
  } else {
    for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) add1(x[c.base + i], t[c.base + i]);
  }
  double r[3] = {(double)a0, (double)a1, (double)a2};
  block_atomic_add<3>(r, acc + 3 * blockIdx.y);
}

// d/dx of the three sums given their gradients g[nc][3] (the target takes no gradient)
__global__ __launch_bounds__(NT) void k_dice_sums_bwd(const float* __restrict__ x, const float* __restrict__ t,
                                                      const float* __restrict__ g, float* __restrict__ dx, int64_t S,
                                                      int flags) {
  const Chunk c = chunk_of(S);
  const float g0 = g[3 * blockIdx.y], g2 = g[3 * blockIdx.y + 2];
  for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) {
    const float xv = x[c.base + i], tv = t[c.base + i];
    const float p = (flags & 1) ? sigm(xv) : xv;
    float d = g0 * tv + ((flags & 2) ? 2.f * g2 * p : g2);
    if (flags & 1) d *= p * (1.f - p);
    dx[c.base + i] = d;
  }
}

// K2: y = prelu((x - mean) * rstd); block (0, nc) also stores mean/rstd for the backward
__global__ __launch_bounds__(NT) void k_in_prelu_apply(const float* __restrict__ x, float* __restrict__ y,
                                                       const double* __restrict__ acc, float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, const float* __restrict__ aw,
                                                       int64_t S, float eps, int vec) {
  const Chunk c = chunk_of(S);
  float mean, rstd;
  stats_of(acc[2 * blockIdx.y], acc[2 * blockIdx.y + 1], S, eps, mean, rstd);
  const float a = *aw;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    mean_out[blockIdx.y] = mean;
    rstd_out[blockIdx.y] = rstd;
  }
  if (vec) {
    const float4* p = reinterpret_cast<const float4*>(x + c.base + c.begin);
    float4* q = reinterpret_cast<float4*>(y + c.base + c.begin);
    const int n4 = (int)((c.end - c.begin) >> 2);
    float4 v[VPT];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = threadIdx.x + k * NT;
      if (i < n4) v[k] = p[i];
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = threadIdx.x + k * NT;
      if (i < n4) {
        float4 o;
        o.x = prelu((v[k].x - mean) * rstd, a);
        o.y = prelu((v[k].y - mean) * rstd, a);
        o.z = prelu((v[k].z - mean) * rstd, a);
        o.w = prelu((v[k].w - mean) * rstd, a);
        q[i] = o;
      }
    }
  } else {
    for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) y[c.base + i] = prelu((x[c.base + i] - mean) * rstd, a);
  }
}

// K3: per-instance sums of g and g*z into acc[nc][2]; sum of dy*z over z<=0 into acc_a[0]
__global__ __launch_bounds__(NT) void k_in_prelu_bwd_stats(const float* __restrict__ x, const float* __restrict__ dy,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in,
                                                           const float* __restrict__ aw, double* __restrict__ acc,
                                                           double* __restrict__ acc_a, int64_t S, int vec) {
  const Chunk c = chunk_of(S);
  const float mean = mean_in[blockIdx.y], rstd = rstd_in[blockIdx.y], a = *aw;
  const double md = mean, rd = rstd;
  // Every sum runs in float64 per thread.  The PReLU weight gradient is one scalar over every voxel
  // of the layer whose terms cancel to 1e-6..1e-8 of their magnitude, and K4's g - mean g - z mean(g z)
  // cancels as deeply where the incoming gradient is nearly affine in z (the top of the U-Net):
  // float32 rounding of z, g z or the partial sums there is what made the step's gradients several
  // times noisier than ATen's (scripts/diag/grad_noise.py).  z is formed in float64 from the stored
  // float32 statistics; the PReLU branch follows the forward's float32 z.
  double s1 = 0.0, s2 = 0.0, sa = 0.0;
  auto visit = [&](float xv, float gv) {
    const bool pos = (xv - mean) * rstd > 0.f;
    const double z = ((double)xv - md) * rd;
    const double g = pos ? (double)gv : (double)a * (double)gv;
    s1 += g;
    s2 += g * z;
    sa += pos ? 0.0 : (double)gv * z;
  };
  if (vec) {
    const float4* px = reinterpret_cast<const float4*>(x + c.base + c.begin);
    const float4* pg = reinterpret_cast<const float4*>(dy + c.base + c.begin);
    const int n4 = (int)((c.end - c.begin) >> 2);
    constexpr int U = VPT / 2;   // two halves keep 2 x 8 float4 in flight
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 vx[U], vg[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int i = threadIdx.x + (h * U + k) * NT;
        const bool ok = i < n4;
        vx[k] = ok ? px[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        vg[k] = ok ? pg[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        visit(vx[k].x, vg[k].x);
        visit(vx[k].y, vg[k].y);
        visit(vx[k].z, vg[k].z);
        visit(vx[k].w, vg[k].w);
      }
    }
  } else {
    for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) visit(x[c.base + i], dy[c.base + i]);
  }
  double r[3] = {s1, s2, sa};
  __shared__ double red[3][NT / 64];
#pragma unroll
  for (int k = 0; k < 3; ++k) r[k] = wave_sum(r[k]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) red[k][wid] = r[k];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[threadIdx.x][w];
    atomicAdd(threadIdx.x < 2 ? &acc[2 * blockIdx.y + threadIdx.x] : acc_a, s);
  }
}

// K4: dx = rstd * (g - mean(g) - z * mean(g z)); block (0,0) also writes the PReLU weight grad
__global__ __launch_bounds__(NT) void k_in_prelu_bwd_apply(const float* __restrict__ x, const float* __restrict__ dy,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in,
                                                           const float* __restrict__ aw,
                                                           const double* __restrict__ acc,
                                                           const double* __restrict__ acc_a, float* __restrict__ dx,
                                                           float* __restrict__ dw, int64_t S, int vec) {
  const Chunk c = chunk_of(S);
  const float mean = mean_in[blockIdx.y], rstd = rstd_in[blockIdx.y], a = *aw;
  const double md = mean, rd = rstd;
  const double mg = acc[2 * blockIdx.y] / (double)S;
  const double mgz = acc[2 * blockIdx.y + 1] / (double)S;
  if (dw && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *dw = (float)(*acc_a);
  auto f = [&](float xv, float gv) {  // float64 combination (see K3): rounded once
    const bool pos = (xv - mean) * rstd > 0.f;
    const double z = ((double)xv - md) * rd;
    const double g = pos ? (double)gv : (double)a * (double)gv;
    return (float)(rd * (g - mg - z * mgz));
  };
  if (vec) {
    const float4* px = reinterpret_cast<const float4*>(x + c.base + c.begin);
    const float4* pg = reinterpret_cast<const float4*>(dy + c.base + c.begin);
    float4* q = reinterpret_cast<float4*>(dx + c.base + c.begin);
    const int n4 = (int)((c.end - c.begin) >> 2);
    constexpr int U = VPT / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 vx[U], vg[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int i = threadIdx.x + (h * U + k) * NT;
        if (i < n4) {
          vx[k] = px[i];
          vg[k] = pg[i];
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int i = threadIdx.x + (h * U + k) * NT;
        if (i < n4) {
          float4 o;
          o.x = f(vx[k].x, vg[k].x);
          o.y = f(vx[k].y, vg[k].y);
          o.z = f(vx[k].z, vg[k].z);
          o.w = f(vx[k].w, vg[k].w);
          q[i] = o;
        }
      }
    }
  } else {
    for (int64_t i = c.begin + threadIdx.x; i < c.end; i += NT) dx[c.base + i] = f(x[c.base + i], dy[c.base + i]);
  }
}

inline bool vec_ok(const void* a, const void* b, const void* c, int64_t S) {
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return S % 4 == 0 && al(a) && al(b) && al(c);
}

}  // namespace

size_t tb_instnorm_prelu_workspace_bytes(int64_t NC) { return (size_t)(2 * NC + 2) * sizeof(double); }

int tb_instnorm_prelu_fwd_f32(const float* x, float* y, float* mean, float* rstd, const float* prelu_w, int64_t NC,
                              int64_t S, float eps, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !y || !mean || !rstd || !prelu_w || !ws || NC < 1 || S < 1 || NC > 65535) return TB_ERR_INVALID_ARG;
  if (ws_bytes < tb_instnorm_prelu_workspace_bytes(NC)) return TB_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* acc = static_cast<double*>(ws);
  const int vec = vec_ok(x, y, nullptr, S) ? 1 : 0;
  const dim3 grid((unsigned)((S + CHUNK - 1) / CHUNK), (unsigned)NC);
  if (hipMemsetAsync(acc, 0, sizeof(double) * 2 * NC, st) != hipSuccess) return TB_ERR_HIP;
  hipLaunchKernelGGL(k_in_stats, grid, dim3(NT), 0, st, x, acc, S, vec);
  hipLaunchKernelGGL(k_in_prelu_apply, grid, dim3(NT), 0, st, x, y, acc, mean, rstd, prelu_w, S, eps, vec);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? TB_OK : TB_ERR_HIP;
}

int tb_instnorm_prelu_bwd_f32(const float* x, const float* dy, const float* mean, const float* rstd,
                              const float* prelu_w, float* dx, float* dw, int64_t NC, int64_t S, void* ws,
                              size_t ws_bytes, void* stream) {
  if (!x || !dy || !mean || !rstd || !prelu_w || !dx || !ws || NC < 1 || S < 1 || NC > 65535)
    return TB_ERR_INVALID_ARG;
  if (ws_bytes < tb_instnorm_prelu_workspace_bytes(NC)) return TB_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* acc = static_cast<double*>(ws);
  double* acc_a = acc + 2 * NC;
  const int vec = vec_ok(x, dy, dx, S) ? 1 : 0;
  const dim3 grid((unsigned)((S + CHUNK - 1) / CHUNK), (unsigned)NC);
  if (hipMemsetAsync(acc, 0, sizeof(double) * (2 * NC + 1), st) != hipSuccess) return TB_ERR_HIP;
  hipLaunchKernelGGL(k_in_prelu_bwd_stats, grid, dim3(NT), 0, st, x, dy, mean, rstd, prelu_w, acc, acc_a, S, vec);
  hipLaunchKernelGGL(k_in_prelu_bwd_apply, grid, dim3(NT), 0, st, x, dy, mean, rstd, prelu_w, acc, acc_a, dx, dw, S,
                     vec);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? TB_OK : TB_ERR_HIP;
}

int tb_channel_sum_f32(const float* x, float* out, int64_t N, int64_t C, int64_t S, void* stream) {
  if (!x || !out || N < 1 || C < 1 || S < 1 || N * C > 65535) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(out, 0, sizeof(float) * (size_t)C, st) != hipSuccess) return TB_ERR_HIP;
  const int vec = (S % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) ? 1 : 0;
  const dim3 grid((unsigned)((S + CHUNK - 1) / CHUNK), (unsigned)(N * C));
  hipLaunchKernelGGL(k_channel_sum, grid, dim3(NT), 0, st, x, out, S, (int)C, vec);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

int tb_dice_sums_f32(const float* x, const float* t, double* sums, int64_t NC, int64_t S, int sigmoid, int squared,
                     void* stream) {
  if (!x || !t || !sums || NC < 1 || S < 1 || NC > 65535) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(sums, 0, sizeof(double) * 3 * (size_t)NC, st) != hipSuccess) return TB_ERR_HIP;
  const int vec = (S % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(t) & 15) == 0);
  const dim3 grid((unsigned)((S + CHUNK - 1) / CHUNK), (unsigned)NC);
  hipLaunchKernelGGL(k_dice_sums, grid, dim3(NT), 0, st, x, t, sums, S, (sigmoid ? 1 : 0) | (squared ? 2 : 0), vec);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

// Dice metric statistics of the reference's evaluation (utils.py:313-411: Activations(sigmoid) +
// AsDiscrete(threshold 0.5), then DiceMetric): per instance {sum t p, sum t, sum p}, p in {0, 1}.
int tb_dice_metric_sums_f32(const float* x, const float* t, double* sums, int64_t NC, int64_t S, void* stream) {
  if (!x || !t || !sums || NC < 1 || S < 1 || NC > 65535) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(sums, 0, sizeof(double) * 3 * (size_t)NC, st) != hipSuccess) return TB_ERR_HIP;
  const int vec = (S % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(t) & 15) == 0);
  const dim3 grid((unsigned)((S + CHUNK - 1) / CHUNK), (unsigned)NC);
  hipLaunchKernelGGL(k_dice_sums, grid, dim3(NT), 0, st, x, t, sums, S, 1 | 4, vec);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

int tb_dice_sums_bwd_f32(const float* x, const float* t, const float* g, float* dx, int64_t NC, int64_t S, int sigmoid,
                         int squared, void* stream) {
  if (!x || !t || !g || !dx || NC < 1 || S < 1 || NC > 65535) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((S + CHUNK - 1) / CHUNK), (unsigned)NC);
  hipLaunchKernelGGL(k_dice_sums_bwd, grid, dim3(NT), 0, st, x, t, g, dx, S, (sigmoid ? 1 : 0) | (squared ? 2 : 0));
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}
