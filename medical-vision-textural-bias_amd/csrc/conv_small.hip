// conv_small.hip -- direct 3x3x3 convolution (stride 1, padding 1) for few channels (Cin, Cout <= 4).
//
// The U-Net the reference trains (MONAI UNet, 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199)
// ends in a full-resolution ResidualUnit(3, 3): a 3 -> 3 Conv3d over 2 x 240 x 240 x 160 voxels.
// With 3 channels the implicit-GEMM library kernels (CK via MIOpen) run at ~1 TFLOP/s (3.5 ms
// forward, 4.8 ms input gradient per step).  The layer is a stencil: each output needs 27 * Cin
// inputs and Cout * 27 * Cin FMAs, so a direct kernel is bound by one HBM sweep of x and y.
//
//   y[n][co][z][h][w] = b[co] + sum_{ci, tz, ty, tx} wt[co][ci][tz][ty][tx] x[n][ci][z+tz-1][h+ty-1][w+tx-1]
//
// The input gradient of the same layer is this convolution of dY with the flipped, transposed
// weights (wt'[ci][co][t] = wt[co][ci][26 - t]), prepared by the caller.
// Block = (n, z, 6 rows of h, all of w): the input tile x[ci][3 tz][8 rows][W + 2] is staged in LDS
// once; each thread owns 4 consecutive w outputs of one row for every co (12 accumulators for
// 3 -> 3), reads 6 inputs per (ci, tz, ty) row and applies 3 tx taps; the weights sit in LDS
// (every lane reads the same address: broadcast).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "texbias.h"
#include "kernels.h"

namespace {

constexpr int NT = 256;
constexpr int ROWS = 6;   // output rows (h) per block
constexpr int WPT = 4;    // consecutive w outputs per thread
constexpr int kSeg = 3;   // 64-lane segments per staged row: XP <= 192

template <int CI, int CO>
__global__ __launch_bounds__(NT) void k_conv3d_small(const float* __restrict__ x, const float* __restrict__ wt,
                                                     const float* __restrict__ bias, float* __restrict__ y, int D,
                                                     int H, int W, int XP, int nhb) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // [CI][3][ROWS + 2][XP], col 0 = w = -1
  static_assert(WPT == 4, "the input reads are one float4 + one float2");
  // weights after the input tile (broadcast LDS reads; 243 of them would spill SGPRs).  No static
  // LDS in this kernel: the dynamic base stays 16-B aligned for the float4 reads.
  float* ws = xs + CI * 3 * (ROWS + 2) * XP;
  const int tid = (int)threadIdx.x;
  for (int i = tid; i < CO * CI * 27; i += NT) ws[i] = wt[i];
  const int hb = (int)blockIdx.x % nhb, z = (int)blockIdx.x / nhb, n = (int)blockIdx.y;
  const int h0 = hb * ROWS;
  const int64_t plane = (int64_t)H * W, vol = (int64_t)D * plane;
  // stage: rows (ci, tz, r) of W floats at column 1, one wave per row (row bounds are scalar);
  // halo columns and out-of-range rows are zero
  constexpr int NR = CI * 3 * (ROWS + 2);
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  static_assert(NR % (NT / 64) == 0, "rows deal evenly to the waves");
#pragma unroll
  for (int row = wave; row < NR; row += NT / 64) {  // fully unrolled: every row's loads in flight
    const int ci = row / (3 * (ROWS + 2)), rem = row - ci * (3 * (ROWS + 2));
    const int tz = rem / (ROWS + 2), r = rem - tz * (ROWS + 2);
    const int zi = z + tz - 1, hi = h0 + r - 1;
    const bool ok = zi >= 0 && zi < D && hi >= 0 && hi < H;
    const float* src = x + ((int64_t)n * CI + ci) * vol + (ok ? (int64_t)zi * plane + (int64_t)hi * W : 0) - 1;
    float* dst = xs + row * XP;
#pragma unroll
    for (int sg = 0; sg < kSeg; ++sg) {
      const int col = lane + 64 * sg;
      const bool in = ok && col >= 1 && col <= W;
      const float v = src[in ? col : 1];
      if (col < XP) dst[col] = in ? v : 0.f;
    }
  }
  __syncthreads();
  const int tpr = (W + WPT - 1) / WPT;  // threads per output row
  const int r = tid / tpr, w0 = (tid - r * tpr) * WPT;
  if (r >= ROWS || h0 + r >= H) return;
  float acc[CO][WPT];
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    const float b = bias ? bias[co] : 0.f;
#pragma unroll
    for (int k = 0; k < WPT; ++k) acc[co][k] = b;
  }
  // (ci, tz) not unrolled: only that slice's 9 * CO weights and 6 inputs per row are live
#pragma unroll 1
  for (int ct = 0; ct < CI * 3; ++ct) {
    const int ci = ct / 3, tz = ct - 3 * ci;
    {
#pragma unroll
      for (int ty = 0; ty < 3; ++ty) {
        const float* src = xs + (ct * (ROWS + 2) + r + ty) * XP + w0;  // column w0 = w0 - 1 + halo
        // 16-B aligned (XP % 4 == 0, w0 % 4 == 0): one ds_read_b128 + one ds_read_b64, no conflicts
        const float4 v4 = *reinterpret_cast<const float4*>(src);
        const float2 v2 = *reinterpret_cast<const float2*>(src + 4);
        const float v[WPT + 2] = {v4.x, v4.y, v4.z, v4.w, v2.x, v2.y};
#pragma unroll
        for (int co = 0; co < CO; ++co) {
#pragma unroll
          for (int tx = 0; tx < 3; ++tx) {
            const float wv = ws[(((co * CI + ci) * 3 + tz) * 3 + ty) * 3 + tx];
#pragma unroll
            for (int k = 0; k < WPT; ++k) acc[co][k] = fmaf(wv, v[k + tx], acc[co][k]);
          }
        }
      }
    }
  }
  const int h = h0 + r;
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    float* dst = y + ((int64_t)n * CO + co) * vol + (int64_t)z * plane + (int64_t)h * W + w0;
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      if (w0 + k < W) dst[k] = acc[co][k];
  }
}

// z-marching form: block = (n, ZB consecutive output planes z, ROWS rows of h).  The input planes
// live in a 4-slot LDS ring ([slot][ci][ROWS + 2 rows][XP]); plane z + 2 is fetched by
// global->LDS DMA (no registers, no waits) while plane z is computed from the slots of z - 1, z,
// z + 1, so every input row is read from memory once per block instead of three times (once per tz
// of each output plane) and its fetch hides under the previous plane's FMAs.
typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
#ifndef TB_SMALL_ZB
#define TB_SMALL_ZB 8
#endif
constexpr int ZB = TB_SMALL_ZB;  // output planes per block

// weights of the z-march as scalar loads from the constant address space (SGPR operands of the packed
// FMAs) instead of per-FMA-group LDS broadcast reads (TB_SMALL_SW=0: LDS): 320 -> 306 us for the C3
// 3 -> 3 layer
#ifndef TB_SMALL_SW
#define TB_SMALL_SW 1
#endif
typedef const __attribute__((address_space(4))) float* cfloat_sp;

// U: (channel, tz) groups unrolled per iteration of the z-march's FMA loop (the weights of a group are
// scalar loads, so a deeper unroll lets more of them be issued ahead; 1 / 3 / 9 measured 280 / 268 / 267 us: 3)
template <int CI, int CO, bool ADD = false, int U = 1>
__global__ __launch_bounds__(NT) void k_conv3d_small_z(const float* __restrict__ x, const float* __restrict__ wt,
                                                       const float* __restrict__ bias, float* __restrict__ y, int D,
                                                       int H, int W, int XP, int nhb, const float* __restrict__ add) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // [4 slots][CI][ROWS + 2][XP], col 0 = w = -1
  constexpr int RS = ROWS + 2, NR = CI * RS;                 // staged rows per plane
  const int slot_f = CI * RS * XP;
  float* ws = xs + 4 * slot_f;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 4 * slot_f; i += NT) xs[i] = 0.f;  // halo columns stay zero (DMA writes 1 .. W)
  for (int i = tid; i < CO * CI * 27; i += NT) ws[i] = wt[i];
  const int hb = (int)blockIdx.x % nhb, z0 = ((int)blockIdx.x / nhb) * ZB, n = (int)blockIdx.y;
  const int h0 = hb * ROWS;
  const int64_t plane = (int64_t)H * W, vol = (int64_t)D * plane;
  __syncthreads();
  // stage input plane zi into ring slot (zi - z0 + 1) & 3: in-range rows by DMA, others zeroed
  auto stage = [&](int zi) {
    float* sl = xs + ((zi - z0 + 1) & 3) * slot_f;
    for (int row = wave; row < NR; row += NT / 64) {
      const int ci = row / RS, r = row - ci * RS, hi = h0 + r - 1;
      float* dst = sl + row * XP + 1;
      if (zi >= 0 && zi < D && hi >= 0 && hi < H) {
        const float* src = x + ((int64_t)n * CI + ci) * vol + (int64_t)zi * plane + (int64_t)hi * W;
#pragma unroll
        for (int sg = 0; sg < kSeg; ++sg) {
          const int c = lane + 64 * sg;
          if (c < W) __builtin_amdgcn_global_load_lds((gptr_t)(src + c), (lptr_t)(dst + 64 * sg), 4, 0, 0);
        }
      } else {
#pragma unroll
        for (int sg = 0; sg < kSeg; ++sg) {
          const int c = lane + 64 * sg;
          if (c < W) dst[c] = 0.f;
        }
      }
    }
  };
  stage(z0 - 1);
  stage(z0);
  stage(z0 + 1);
  __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA landed
  __syncthreads();
  const int tpr = (W + WPT - 1) / WPT;
  const int r = tid / tpr, w0 = (tid - r * tpr) * WPT;
  const bool act = r < ROWS && h0 + r < H;
  const int zend = z0 + ZB < D ? z0 + ZB : D;
  const int h = h0 + r;
  // step z: fetch plane z + 2 | store step z - 1's outputs | FMAs of plane z into registers | wait, barrier.
  // The outputs leave one step late, so the wait for the fetch never waits for the step's own stores
  // (the residual `add` values are loaded at the start of their step, used a step later).
  float prev[CO][WPT], padd[CO][WPT];
  auto put = [&](int zp) {
#pragma unroll
    for (int co = 0; co < CO; ++co) {
      const int64_t o = ((int64_t)n * CO + co) * vol + (int64_t)zp * plane + (int64_t)h * W + w0;
#pragma unroll
      for (int k = 0; k < WPT; ++k)
        if (w0 + k < W) y[o + k] = ADD ? prev[co][k] + padd[co][k] : prev[co][k];
    }
  };
  for (int z = z0; z < zend; ++z) {
    if (z + 2 < zend + 1) stage(z + 2);  // the next plane's fetch overlaps this plane's FMAs
    if (act) {
      if (z > z0) put(z - 1);
      if (ADD) {
#pragma unroll
        for (int co = 0; co < CO; ++co) {
          const int64_t o = ((int64_t)n * CO + co) * vol + (int64_t)z * plane + (int64_t)h * W + w0;
#pragma unroll
          for (int k = 0; k < WPT; ++k) padd[co][k] = w0 + k < W ? add[o + k] : 0.f;
        }
      }
      float acc[CO][WPT];
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        const float b = bias ? bias[co] : 0.f;
#pragma unroll
        for (int k = 0; k < WPT; ++k) acc[co][k] = b;
      }
#pragma unroll U
      for (int ct = 0; ct < CI * 3; ++ct) {
        const int ci = ct / 3, tz = ct - 3 * ci;
        const float* base = xs + ((z - z0 + tz) & 3) * slot_f + (ci * RS + r) * XP + w0;
#pragma unroll
        for (int ty = 0; ty < 3; ++ty) {
          const float* src = base + ty * XP;
          const float4 v4 = *reinterpret_cast<const float4*>(src);
          const float2 v2 = *reinterpret_cast<const float2*>(src + 4);
          const float v[WPT + 2] = {v4.x, v4.y, v4.z, v4.w, v2.x, v2.y};
#pragma unroll
          for (int co = 0; co < CO; ++co) {
#pragma unroll
            for (int tx = 0; tx < 3; ++tx) {
              const int wi = (((co * CI + ci) * 3 + tz) * 3 + ty) * 3 + tx;
              const float wv = TB_SMALL_SW ? ((cfloat_sp)wt)[wi] : ws[wi];
#pragma unroll
              for (int k = 0; k < WPT; ++k) acc[co][k] = fmaf(wv, v[k + tx], acc[co][k]);
            }
          }
        }
      }
#pragma unroll
      for (int co = 0; co < CO; ++co)
#pragma unroll
        for (int k = 0; k < WPT; ++k) prev[co][k] = acc[co][k];
    }
    __builtin_amdgcn_s_waitcnt(0);  // plane z + 2 landed (this wave's share; the stores were issued a step ago)
    __syncthreads();                // ... and every wave's; slot of z - 1 free for plane z + 3
  }
  if (act && zend > z0) put(zend - 1);
}

__global__ __launch_bounds__(256) void k_add_inplace(float* __restrict__ y, const float* __restrict__ a, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] += a[i];
}

template <int CI, int CO>
int launch(const float* x, const float* w, const float* b, const float* add, float* y, int N, int D, int H, int W,
           hipStream_t st) {
  const int XP = (W + 2 + WPT + 3) / 4 * 4;  // halo, slack for the last thread's 6-wide read, 16-B rows
  const size_t lds = sizeof(float) * ((size_t)CI * 3 * (ROWS + 2) * XP + CO * CI * 27);
  if ((W + WPT - 1) / WPT * ROWS > NT || lds > 65536 || XP > 64 * kSeg) return TB_ERR_UNSUPPORTED_SIZE;
  const int nhb = (H + ROWS - 1) / ROWS;
  const size_t lds_z = sizeof(float) * ((size_t)4 * CI * (ROWS + 2) * XP + CO * CI * 27);
  if (lds_z <= 65536 * 2) {  // z-march (3 (channel, tz) groups per FMA-loop iteration)
    void (*kern)(const float*, const float*, const float*, float*, int, int, int, int, int, const float*) =
        add ? k_conv3d_small_z<CI, CO, true, 3> : k_conv3d_small_z<CI, CO, false, 3>;
    if (tb::allow_full_lds(kern) != hipSuccess) return TB_ERR_HIP;  // once per kernel (kernels.h)
    hipLaunchKernelGGL(kern, dim3((unsigned)(nhb * ((D + ZB - 1) / ZB)), (unsigned)N), dim3(NT), lds_z, st, x, w, b, y,
                       D, H, W, XP, nhb, add);
    return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
  }
  hipLaunchKernelGGL((k_conv3d_small<CI, CO>), dim3((unsigned)(nhb * D), (unsigned)N), dim3(NT), lds, st, x, w, b, y,
                     D, H, W, XP, nhb);
  if (add) {  // the plane-per-block kernel has no residual epilogue: a separate y += add pass
    const int64_t n = (int64_t)N * CO * D * H * W;
    hipLaunchKernelGGL(k_add_inplace, dim3((unsigned)((n + 1023) / 1024 < 8192 ? (n + 1023) / 1024 : 8192)), dim3(256),
                       0, st, y, add, n);
  }
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

}  // namespace

int tb_conv3d_small_f32(const float* x, const float* w, const float* b, float* y, int N, int Cin, int Cout, int D,
                        int H, int W, void* stream) {
  return tb_conv3d_small_add_f32(x, w, b, nullptr, y, N, Cin, Cout, D, H, W, stream);
}

int tb_conv3d_small_add_f32(const float* x, const float* w, const float* b, const float* add, float* y, int N, int Cin,
                            int Cout, int D, int H, int W, void* stream) {
  if (!x || !w || !y || N < 1 || D < 1 || H < 1 || W < 1 || N > 65535) return TB_ERR_INVALID_ARG;
  if (Cin < 1 || Cin > 4 || Cout < 1 || Cout > 4) return TB_ERR_UNSUPPORTED_SIZE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define TB_CASE(ci, co) \
  if (Cin == ci && Cout == co) return launch<ci, co>(x, w, b, add, y, N, D, H, W, st);
#define TB_ROW(ci) TB_CASE(ci, 1) TB_CASE(ci, 2) TB_CASE(ci, 3) TB_CASE(ci, 4)
  TB_ROW(1) TB_ROW(2) TB_ROW(3) TB_ROW(4)
#undef TB_ROW
#undef TB_CASE
  return TB_ERR_UNSUPPORTED_SIZE;
}
