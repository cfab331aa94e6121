// optim.hip -- the train step's Adam update (torch.optim.Adam(lr, weight_decay, amsgrad) as the reference
// configures it: 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:203-205, Adam(model.parameters(), 1e-4,
// weight_decay=1e-5, amsgrad=True)) over every parameter tensor in one launch.
//
// ATen's fused Adam runs the U-Net's ~4.8 M parameters as three multi-tensor launches of 40 / 84 / 3
// blocks (one 64 K-element chunk per block): 112 us per step at ~1.2 TB/s, since 84 blocks cannot fill
// 256 CUs.  Here the tensors are cut into 4096-element chunks (~1200 blocks), each block finds its
// tensor in the launch's table (kernel argument, up to 32 tensors per launch) and streams p, g, m, v,
// vmax as float4: 28 B read + 16 B written per element (amsgrad), HBM-bound.
//
// Per element, the expressions and types of ATen's fused Adam (ADAM_MODE::ORIGINAL: the hyper-parameters
// are doubles, the state float32, each statement rounded to float32 once):
//   g <- g + p wd;  m <- b1 m + (1 - b1) g;  v <- b2 v + (1 - b2) g g;  vmax <- max(vmax, v)
//   p <- p - (lr / bc1) m / (sqrt(vmax) / sqrt(bc2) + eps),  bc1 = 1 - b1^t, bc2 = 1 - b2^t (float32)
// (v instead of vmax without amsgrad)
// with t the tensor's step count, read from the device (incremented by the caller before the launch, as
// torch's fused / capturable Adam keeps it), so the update is graph-capturable.
#include <hip/hip_runtime.h>

#include <cmath>

#include "texbias.h"

namespace {

constexpr int ANT = 256;             // threads per block
constexpr int AVP = 4;               // float4 per thread per array
constexpr int ACH = ANT * AVP * 4;   // elements per chunk
constexpr int AMAXT = 32;            // tensors per launch

struct AdamTab {
  float* p[AMAXT];
  const float* g[AMAXT];
  float* m[AMAXT];
  float* v[AMAXT];
  float* vmax[AMAXT];
  const float* step[AMAXT];
  int64_t n[AMAXT];
  int c0[AMAXT + 1];  // first chunk of each tensor; c0[nt] = chunks of the launch
  int nt, amsgrad, vec_mask;  // vec_mask bit i: tensor i is 16-B aligned with numel % 4 == 0
  double lr, b1, b2, eps, wd;
};

struct AdamCoef {
  float step_size, bc2_sqrt;
};

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float* vmax, const AdamTab& t,
                                      const AdamCoef& c) {
  if (t.wd != 0.0) g = (float)((double)g + (double)p * t.wd);
  m = (float)(t.b1 * (double)m + (1.0 - t.b1) * (double)g);
  v = (float)(t.b2 * (double)v + (1.0 - t.b2) * (double)g * (double)g);
  float d = v;
  if (vmax) {
    d = fmaxf(*vmax, v);
    *vmax = d;
  }
  const float denom = (float)((double)(sqrtf(d) / c.bc2_sqrt) + t.eps);
  p -= c.step_size * m / denom;
}

__global__ __launch_bounds__(ANT) void k_adam(const AdamTab t) {
  const int chunk = (int)blockIdx.x;
  int i = 0;
  while (i + 1 < t.nt && chunk >= t.c0[i + 1]) ++i;
  const int64_t b = (int64_t)(chunk - t.c0[i]) * ACH;
  const int64_t e = b + ACH < t.n[i] ? b + ACH : t.n[i];
  const double st = (double)*t.step[i];
  const float bc1 = (float)(1.0 - pow(t.b1, st));
  AdamCoef c;
  c.step_size = (float)(t.lr / (double)bc1);
  c.bc2_sqrt = (float)sqrt(1.0 - pow(t.b2, st));
  float* P = t.p[i] + b;
  const float* G = t.g[i] + b;
  float* M = t.m[i] + b;
  float* V = t.v[i] + b;
  float* X = t.amsgrad ? t.vmax[i] + b : nullptr;
  const int len = (int)(e - b);
  if ((t.vec_mask >> i) & 1) {
    const int n4 = len >> 2;
    float4 pv[AVP], gv[AVP], mv[AVP], vv[AVP], xv[AVP];
#pragma unroll
    for (int k = 0; k < AVP; ++k) {  // every load issued before the first use (indices clamped)
      const int j = (int)threadIdx.x + k * ANT, jj = j < n4 ? j : n4 - 1;
      pv[k] = reinterpret_cast<const float4*>(P)[jj];
      gv[k] = reinterpret_cast<const float4*>(G)[jj];
      mv[k] = reinterpret_cast<const float4*>(M)[jj];
      vv[k] = reinterpret_cast<const float4*>(V)[jj];
      if (X) xv[k] = reinterpret_cast<const float4*>(X)[jj];
    }
#pragma unroll
    for (int k = 0; k < AVP; ++k) {
      const int j = (int)threadIdx.x + k * ANT;
      if (j >= n4) continue;
      float* xs = X ? &xv[k].x : nullptr;
      adam1(pv[k].x, gv[k].x, mv[k].x, vv[k].x, xs, t, c);
      adam1(pv[k].y, gv[k].y, mv[k].y, vv[k].y, X ? &xv[k].y : nullptr, t, c);
      adam1(pv[k].z, gv[k].z, mv[k].z, vv[k].z, X ? &xv[k].z : nullptr, t, c);
      adam1(pv[k].w, gv[k].w, mv[k].w, vv[k].w, X ? &xv[k].w : nullptr, t, c);
      reinterpret_cast<float4*>(P)[j] = pv[k];
      reinterpret_cast<float4*>(M)[j] = mv[k];
      reinterpret_cast<float4*>(V)[j] = vv[k];
      if (X) reinterpret_cast<float4*>(X)[j] = xv[k];
    }
  } else {
    for (int j = (int)threadIdx.x; j < len; j += ANT) {
      float p = P[j], m = M[j], v = V[j];
      adam1(p, G[j], m, v, X ? X + j : nullptr, t, c);
      P[j] = p, M[j] = m, V[j] = v;
    }
  }
}

}  // namespace

int tb_adam_f32(int nt, float* const* param, const float* const* grad, float* const* exp_avg,
                float* const* exp_avg_sq, float* const* max_exp_avg_sq, const float* const* step,
                const int64_t* numel, double lr, double beta1, double beta2, double eps, double weight_decay,
                int amsgrad, void* stream) {
  if (nt < 0 || (nt > 0 && (!param || !grad || !exp_avg || !exp_avg_sq || !step || !numel)) ||
      (amsgrad && nt > 0 && !max_exp_avg_sq))
    return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  for (int t0 = 0; t0 < nt; t0 += AMAXT) {
    AdamTab a{};
    a.nt = 0, a.amsgrad = amsgrad ? 1 : 0;
    a.lr = lr, a.b1 = beta1, a.b2 = beta2, a.eps = eps, a.wd = weight_decay;
    int chunks = 0;
    for (int k = t0; k < nt && k < t0 + AMAXT; ++k) {
      if (numel[k] < 0 || numel[k] > (int64_t)ACH * (1 << 20)) return TB_ERR_INVALID_ARG;
      if (numel[k] == 0) continue;
      if (!param[k] || !grad[k] || !exp_avg[k] || !exp_avg_sq[k] || !step[k] || (amsgrad && !max_exp_avg_sq[k]))
        return TB_ERR_INVALID_ARG;
      const int i = a.nt++;
      a.p[i] = param[k], a.g[i] = grad[k], a.m[i] = exp_avg[k], a.v[i] = exp_avg_sq[k];
      a.vmax[i] = amsgrad ? max_exp_avg_sq[k] : nullptr;
      a.step[i] = step[k], a.n[i] = numel[k];
      a.c0[i] = chunks;
      chunks += (int)((numel[k] + ACH - 1) / ACH);
      const bool vec = numel[k] % 4 == 0 && al16(param[k]) && al16(grad[k]) && al16(exp_avg[k]) &&
                       al16(exp_avg_sq[k]) && (!amsgrad || al16(max_exp_avg_sq[k]));
      if (vec) a.vec_mask |= 1 << i;
    }
    a.c0[a.nt] = chunks;
    if (a.nt == 0) continue;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)chunks), dim3(ANT), 0, st, a);
    if (hipGetLastError() != hipSuccess) return TB_ERR_HIP;
  }
  return TB_OK;
}
