// prep.hip -- GPU-side BraTS preprocessing of a batch of resident raw volumes.
//
// The reference's training Compose runs these per sample in CPU DataLoader workers before the
// texture filters (10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
// stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:151-170):
//   ConvertToMultiChannelBasedOnBratsClassesd  source_code/filters_and_operators.py:61-87
//   RandSpatialCropd(roi)                      MONAI 0.5: slice at a host-drawn corner
//   RandFlipd(prob, spatial_axis)              MONAI 0.5: np.flip per channel
//   NormalizeIntensityd(nonzero, channel_wise) MONAI 0.5: (x - mean) / std over x != 0, per channel
//   RandScaleIntensityd(factors, prob)         MONAI 0.5: x * (1 + factor)
//   RandShiftIntensityd(offsets, prob)         MONAI 0.5: x + offset (every voxel)
// Here: one statistics pass over each (sample, channel) crop window (nonzero count, sum, sum of
// squares in float64; per-chunk partials, no atomics), a finalize pass folding the three
// intensity transforms into y = x != 0 ? a x + b : g per (sample, channel), and one gather pass
// writing the cropped, flipped, normalised image and the 3-channel label together.  HBM traffic:
// the crop window read twice (stats, apply) + the output written once.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "texbias.h"

namespace {

constexpr int PNT = 256;
constexpr int PCHUNK = 64;  // statistics partials per (sample, channel)

struct PrepArgs {
  const float* img;
  const float* lab;
  int C, H0, W0, D0, h, w, d;
  int64_t isb, isc;  // input strides (elements) of sample / channel
  int64_t lsb;       // label sample stride
  float* out;
  float* olab;
  double* part;  // [B C][PCHUNK][3]
  float* coef;   // [B C][3]: a, b, g
  tb_prep_params p[TB_MAX_BATCH];
};

__device__ __forceinline__ const float* row_src(const PrepArgs& a, const tb_prep_params& q, const float* base, int i,
                                                int j) {
  // output row (i, j) of the crop -> input row, with the flips applied inside the window
  const int si = q.flip & 1 ? a.h - 1 - i : i;
  const int sj = q.flip & 2 ? a.w - 1 - j : j;
  return base + ((int64_t)(q.h0 + si) * a.W0 + (q.w0 + sj)) * a.D0 + q.d0;
}

// Resample mode: the input coordinate of output voxel (i, j, k) under the sample's 3 x 4 map.
struct Coord3 {
  float x, y, z;
};
__device__ __forceinline__ Coord3 map_row(const tb_prep_params& q, int i, int j) {
  return Coord3{fmaf(q.m[0], (float)i, fmaf(q.m[1], (float)j, q.m[3])),
                fmaf(q.m[4], (float)i, fmaf(q.m[5], (float)j, q.m[7])),
                fmaf(q.m[8], (float)i, fmaf(q.m[9], (float)j, q.m[11]))};
}
__device__ __forceinline__ Coord3 map_at(const tb_prep_params& q, const Coord3& r, int k) {
  return Coord3{fmaf(q.m[2], (float)k, r.x), fmaf(q.m[6], (float)k, r.y), fmaf(q.m[10], (float)k, r.z)};
}
// one axis of the border-clamped trilinear stencil: (i0, i1, weight of i1)
__device__ __forceinline__ void axis_lin(float c, int n, int& i0, int& i1, float& f) {
  c = fminf(fmaxf(c, 0.f), (float)(n - 1));
  const float fl = floorf(c);
  i0 = (int)fl;
  i1 = i0 + 1 < n ? i0 + 1 : n - 1;
  f = c - fl;
}
__device__ __forceinline__ float trilinear(const float* v, const PrepArgs& a, const Coord3& c) {
  int x0, x1, y0, y1, z0, z1;
  float fx, fy, fz;
  axis_lin(c.x, a.H0, x0, x1, fx);
  axis_lin(c.y, a.W0, y0, y1, fy);
  axis_lin(c.z, a.D0, z0, z1, fz);
  auto at = [&](int x, int y, int z) { return v[((int64_t)x * a.W0 + y) * a.D0 + z]; };
  const float c00 = fmaf(fz, at(x0, y0, z1) - at(x0, y0, z0), at(x0, y0, z0));
  const float c01 = fmaf(fz, at(x0, y1, z1) - at(x0, y1, z0), at(x0, y1, z0));
  const float c10 = fmaf(fz, at(x1, y0, z1) - at(x1, y0, z0), at(x1, y0, z0));
  const float c11 = fmaf(fz, at(x1, y1, z1) - at(x1, y1, z0), at(x1, y1, z0));
  const float c0 = fmaf(fy, c01 - c00, c00), c1 = fmaf(fy, c11 - c10, c10);
  return fmaf(fx, c1 - c0, c0);
}
__device__ __forceinline__ int axis_near(float c, int n) {
  const int i = (int)rintf(c);  // round half to even (grid_sample's nearbyint)
  return i < 0 ? 0 : (i >= n ? n - 1 : i);
}
__device__ __forceinline__ float nearest(const float* v, const PrepArgs& a, const Coord3& c) {
  return v[((int64_t)axis_near(c.x, a.H0) * a.W0 + axis_near(c.y, a.W0)) * a.D0 + axis_near(c.z, a.D0)];
}

__global__ __launch_bounds__(PNT) void k_prep_stats(PrepArgs a) {
  __shared__ double red[3][PNT / 64];
  const int bc = (int)blockIdx.y, b = bc / a.C, c = bc - b * a.C;
  const tb_prep_params& q = a.p[b];
  const float* base = a.img + b * a.isb + c * a.isc;
  const int rows = a.h * a.w;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double s = 0.0, s2 = 0.0, n = 0.0;
  for (int r = (int)blockIdx.x * (PNT / 64) + wid; r < rows; r += PCHUNK * (PNT / 64)) {  // a row per wave
    const int i = r / a.w, j = r - i * a.w;
    if (q.resample) {
      const Coord3 rb = map_row(q, i, j);
      for (int k = lane; k < a.d; k += 64) {
        const float v = trilinear(base, a, map_at(q, rb, k));
        if (v != 0.f) {
          s += v;
          s2 += (double)v * v;
          n += 1.0;
        }
      }
      continue;
    }
    const float* src = row_src(a, q, base, i, j);
    for (int k = lane; k < a.d; k += 64) {
      const float v = src[k];
      if (v != 0.f) {
        s += v;
        s2 += (double)v * v;
        n += 1.0;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    s2 += __shfl_xor(s2, o);
    n += __shfl_xor(n, o);
  }
  if (lane == 0) {
    red[0][wid] = s;
    red[1][wid] = s2;
    red[2][wid] = n;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double t = 0.0;
    for (int k = 0; k < PNT / 64; ++k) t += red[threadIdx.x][k];
    a.part[((int64_t)bc * PCHUNK + blockIdx.x) * 3 + threadIdx.x] = t;
  }
}

__global__ void k_prep_finalize(PrepArgs a, int nbc) {
  const int bc = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (bc >= nbc) return;
  const tb_prep_params& q = a.p[bc / a.C];
  double s = 0.0, s2 = 0.0, n = 0.0;
  for (int k = 0; k < PCHUNK; ++k) {
    const double* t = a.part + ((int64_t)bc * PCHUNK + k) * 3;
    s += t[0];
    s2 += t[1];
    n += t[2];
  }
  float mean = 0.f, sd = 1.f;
  if (q.normalize && n > 0.0) {
    const double m = s / n;
    const double var = s2 / n - m * m;
    mean = (float)m;
    sd = (float)sqrt(var > 0.0 ? var : 0.0);
    if (sd == 0.f) sd = 1.f;  // MONAI: a zero std divides by 1
  }
  const float sc = q.scale, sh = q.shift;
  float* co = a.coef + (int64_t)bc * 3;
  if (q.normalize && n > 0.0) {
    co[0] = sc / sd;
    co[1] = sh - sc * mean / sd;
  } else {
    co[0] = sc;
    co[1] = sh;
  }
  co[2] = sh;  // zero voxels: only the shift reaches them
}

__global__ __launch_bounds__(PNT) void k_prep_apply(PrepArgs a, int B) {
  const int nrow = a.h * a.w;
  const int64_t nimg = (int64_t)B * a.C * nrow;  // image rows, then label rows (one per sample row)
  const int64_t nlab = a.olab ? (int64_t)B * nrow : 0;
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (PNT / 64) + (threadIdx.x >> 6); r < nimg + nlab;
       r += (int64_t)gridDim.x * (PNT / 64)) {  // a row per wave
    if (r < nimg) {
      const int64_t bc = r / nrow;
      const int rr = (int)(r - bc * nrow), i = rr / a.w, j = rr - i * a.w;
      const int b = (int)(bc / a.C), c = (int)(bc - (int64_t)b * a.C);
      const float ca = a.coef[bc * 3], cb = a.coef[bc * 3 + 1], cg = a.coef[bc * 3 + 2];
      float* dst = a.out + r * a.d;
      if (a.p[b].resample) {
        const float* base = a.img + b * a.isb + c * a.isc;
        const Coord3 rb = map_row(a.p[b], i, j);
        for (int k = lane; k < a.d; k += 64) {
          const float v = trilinear(base, a, map_at(a.p[b], rb, k));
          dst[k] = v != 0.f ? fmaf(ca, v, cb) : cg;
        }
        continue;
      }
      const float* src = row_src(a, a.p[b], a.img + b * a.isb + c * a.isc, i, j);
      const bool fd = a.p[b].flip & 4;
      for (int k = lane; k < a.d; k += 64) {
        const float v = src[fd ? a.d - 1 - k : k];
        dst[k] = v != 0.f ? fmaf(ca, v, cb) : cg;
      }
    } else {
      const int64_t lr = r - nimg;
      const int b = (int)(lr / nrow);
      const int rr = (int)(lr - (int64_t)b * nrow), i = rr / a.w, j = rr - i * a.w;
      const bool rs = a.p[b].resample;
      const float* src = rs ? a.lab + b * a.lsb : row_src(a, a.p[b], a.lab + b * a.lsb, i, j);
      const Coord3 rb = rs ? map_row(a.p[b], i, j) : Coord3{0.f, 0.f, 0.f};
      const int64_t plane = (int64_t)nrow * a.d;
      float* dst = a.olab + (int64_t)b * 3 * plane + (int64_t)rr * a.d;
      const bool fd = a.p[b].flip & 4;
      for (int k = lane; k < a.d; k += 64) {
        const float v = rs ? nearest(src, a, map_at(a.p[b], rb, k)) : src[fd ? a.d - 1 - k : k];
        const bool l1 = v == 1.f, l2 = v == 2.f, l3 = v == 3.f;
        dst[k] = (l2 || l3) ? 1.f : 0.f;             // TC: labels 2, 3
        dst[plane + k] = (l1 || l2 || l3) ? 1.f : 0.f;  // WT: labels 1, 2, 3
        dst[2 * plane + k] = l2 ? 1.f : 0.f;           // ET: label 2
      }
    }
  }
}

}  // namespace

size_t tb_brats_prep_workspace_bytes(int B, int C) {
  return (size_t)B * C * (PCHUNK * 3 * sizeof(double) + 4 * sizeof(float)) + 256;
}

int tb_brats_prep_f32(const float* img, const float* lab, int B, int C, int H0, int W0, int D0,
                      const tb_prep_params* params, int h, int w, int d, float* out, float* out_lab, void* ws,
                      size_t ws_bytes, void* stream) {
  if (!img || !params || !out || B < 1 || C < 1 || H0 < 1 || W0 < 1 || D0 < 1 || h < 1 || w < 1 || d < 1)
    return TB_ERR_INVALID_ARG;
  bool crop_only = true;
  for (int b = 0; b < B; ++b) crop_only &= params[b].resample == 0;
  if (crop_only && (h > H0 || w > W0 || d > D0)) return TB_ERR_INVALID_ARG;
  if (out_lab && !lab) return TB_ERR_INVALID_ARG;
  if (!ws || ws_bytes < tb_brats_prep_workspace_bytes(B < TB_MAX_BATCH ? B : TB_MAX_BATCH, C))
    return TB_ERR_WORKSPACE;
  for (int b = 0; b < B; ++b) {
    const tb_prep_params& q = params[b];
    if (q.resample) {  // any finite map: the sampling clamps to the volume
      for (int e = 0; e < 12; ++e)
        if (!std::isfinite(q.m[e])) return TB_ERR_INVALID_ARG;
      continue;
    }
    if (q.h0 < 0 || q.w0 < 0 || q.d0 < 0 || q.h0 + h > H0 || q.w0 + w > W0 || q.d0 + d > D0 || (q.flip & ~7))
      return TB_ERR_INVALID_ARG;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t isc = (int64_t)H0 * W0 * D0, isb = isc * C;
  const int64_t osb = (int64_t)C * h * w * d, olb = 3LL * h * w * d;
  for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
    const int nb = B - b0 < TB_MAX_BATCH ? B - b0 : TB_MAX_BATCH;
    PrepArgs a{};
    a.img = img + b0 * isb;
    a.lab = lab ? lab + b0 * (int64_t)H0 * W0 * D0 : nullptr;
    a.C = C; a.H0 = H0; a.W0 = W0; a.D0 = D0; a.h = h; a.w = w; a.d = d;
    a.isb = isb; a.isc = isc; a.lsb = (int64_t)H0 * W0 * D0;
    a.out = out + b0 * osb;
    a.olab = out_lab ? out_lab + b0 * olb : nullptr;
    a.part = reinterpret_cast<double*>(ws);
    a.coef = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + (size_t)nb * C * PCHUNK * 3 * sizeof(double));
    for (int i = 0; i < nb; ++i) a.p[i] = params[b0 + i];
    const int nbc = nb * C;
    hipLaunchKernelGGL(k_prep_stats, dim3(PCHUNK, nbc), dim3(PNT), 0, st, a);
    if (hipGetLastError() != hipSuccess) return TB_ERR_HIP;
    hipLaunchKernelGGL(k_prep_finalize, dim3((nbc + 63) / 64), dim3(64), 0, st, a, nbc);
    if (hipGetLastError() != hipSuccess) return TB_ERR_HIP;
    const int64_t rows = (int64_t)nb * (C + (out_lab ? 1 : 0)) * h * w;
    const int grid = (int)((rows + 3) / 4 < 8192 ? (rows + 3) / 4 : 8192);
    hipLaunchKernelGGL(k_prep_apply, dim3(grid), dim3(PNT), 0, st, a, nb);
    if (hipGetLastError() != hipSuccess) return TB_ERR_HIP;
  }
  return TB_OK;
}
