// conv_wgrad.hip -- 3-D convolution weight gradient (f32, MFMA 16x16x4) for the U-Net train step.
//
// The reference trains MONAI's 3-D U-Net (10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-204)
// and its backward needs dW of every Conv3d / ConvTranspose3d.  MIOpen on gfx950 runs the
// weight gradient of the full-resolution layers (K = N * 120*120*80 = 2.3 M reduction positions,
// only 16 x 16 x 27 outputs) with a naive kernel or a CK GEMM without split-K: ~350 ms each.
// This kernel is a split-K implicit GEMM:
//   dW[m][c][tz][ty][tx] = sum_n sum_{z,y,x} G[n][m][z][y][x] * X[n][c][s z + tz - p][s y + ty - p][s x + tx - p]
// which covers both layer kinds:
//   Conv3d          : G = dY [N][Cout][out],  X = x  [N][Cin][in],   dW = [Cout][Cin][k^3]
//   ConvTranspose3d : G = x  [N][Cin][in],    X = dY [N][Cout][out], dW = [Cin][Cout][k^3]
// (PyTorch's transposed conv places x[q] at s q - p + t, the same index map).
//
// Work split: blockIdx.y = (16-row m tile, 16-col c tile); blockIdx.x strides over "chunks" =
// (n, z, y, x-segment of XT outputs).  Per chunk the block stages G[16][XT] and the 3x3 (tz,ty)
// input rows X[16][9][s(XT-1)+3] in LDS; each of the 4 waves owns 7 (or 6) of the 27 taps and
// runs v_mfma_f32_16x16x4_f32 over the chunk's positions (K = 4 per instruction, exact f32 FMA
// chains).  Partial sums leave the block once, by float atomics into dW (zeroed first).
#include <hip/hip_runtime.h>

#include "texbias.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int S, int XT>
struct WgGeo {
  static constexpr int GP = XT + 1;                // padded G row (bank spread)
  static constexpr int XS = S * (XT - 1) + 3;      // input row span per chunk
  static constexpr int XP = XS | 1;                // odd pitch
  static constexpr int ROWS = 9;                   // (tz, ty)
};

template <int S, int XT>
__global__ __launch_bounds__(256) void k_conv3d_wgrad(const float* __restrict__ G, const float* __restrict__ X,
                                                      float* __restrict__ dW, int M, int Cc, int Do, int Ho, int Wo,
                                                      int Di, int Hi, int Wi, int pad, int nxt, int64_t nchunks,
                                                      int ctiles) {
  using Gm = WgGeo<S, XT>;
  __shared__ float gs[16 * Gm::GP];
  __shared__ float xs[16 * Gm::ROWS * Gm::XP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mt = blockIdx.y / ctiles, ct = blockIdx.y - mt * ctiles;
  const int m0 = mt * 16, c0 = ct * 16;
  const int mv = min(16, M - m0), cv = min(16, Cc - c0);
  const int64_t gstride_m = (int64_t)Do * Ho * Wo, xstride_c = (int64_t)Di * Hi * Wi;
  f32x4 acc[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    int64_t r = ch;
    const int xt = (int)(r % nxt); r /= nxt;
    const int y = (int)(r % Ho); r /= Ho;
    const int z = (int)(r % Do);
    const int n = (int)(r / Do);
    const int x0 = xt * XT;
    // stage G[m][x0 .. x0+XT)
    const float* gb = G + ((int64_t)n * M + m0) * gstride_m + ((int64_t)z * Ho + y) * Wo;
    for (int i = tid; i < 16 * XT; i += 256) {
      const int m = i / XT, xx = i - m * XT;
      float v = 0.f;
      if (m < mv && x0 + xx < Wo) v = gb[(int64_t)m * gstride_m + x0 + xx];
      gs[m * Gm::GP + xx] = v;
    }
    // stage X[c][(tz,ty)][S*x0 - pad + j], j < XS
    const int xin0 = S * x0 - pad;
    const float* xb = X + ((int64_t)n * Cc + c0) * xstride_c;
    const int nx = cv * Gm::ROWS * Gm::XS;
    for (int i = tid; i < 16 * Gm::ROWS * Gm::XS; i += 256) {
      float v = 0.f;
      const int c = i / (Gm::ROWS * Gm::XS);
      const int rem = i - c * (Gm::ROWS * Gm::XS);
      const int row = rem / Gm::XS, j = rem - row * Gm::XS;
      if (i < nx) {
        const int zi = S * z + row / 3 - pad, yi = S * y + row % 3 - pad, xi = xin0 + j;
        if (zi >= 0 && zi < Di && yi >= 0 && yi < Hi && xi >= 0 && xi < Wi)
          v = xb[(int64_t)c * xstride_c + ((int64_t)zi * Hi + yi) * Wi + xi];
      }
      xs[(c * Gm::ROWS + row) * Gm::XP + j] = v;
    }
    __syncthreads();
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
    for (int kk = 0; kk < XT; kk += 4) {
      const float a = gs[li * Gm::GP + kk + lk];
      const int xoff = S * (kk + lk);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const int t = wave + 4 * j;
        if (t < 27) {
          const int row = t / 3, tx = t - 3 * row;   // t = (tz*3 + ty)*3 + tx
          const float b = xs[(li * Gm::ROWS + row) * Gm::XP + xoff + tx];
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // D[row = m][col = c]: lane holds rows (lane>>4)*4 + r, col lane & 15
  const int c = lane & 15;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int t = wave + 4 * j;
    if (t >= 27 || c >= cv) continue;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = (lane >> 4) * 4 + rr;
      if (m < mv) atomicAdd(&dW[((int64_t)(m0 + m) * Cc + (c0 + c)) * 27 + t], acc[j][rr]);
    }
  }
}

template <int S, int XT>
int launch(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi,
           int Wi, int pad, hipStream_t st) {
  const int nxt = (Wo + XT - 1) / XT;
  const int64_t nchunks = (int64_t)N * Do * Ho * nxt;
  const int mtiles = (M + 15) / 16, ctiles = (Cc + 15) / 16;
  // enough blocks to fill the chip ~4x over, never more than there are chunks
  int64_t gx = (2048 + mtiles * ctiles - 1) / (mtiles * ctiles);
  if (gx > nchunks) gx = nchunks;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((k_conv3d_wgrad<S, XT>), dim3((unsigned)gx, mtiles * ctiles), dim3(256), 0, st, G, X, dW, M,
                     Cc, Do, Ho, Wo, Di, Hi, Wi, pad, nxt, nchunks, ctiles);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

}  // namespace

// dW (M x Cc x 27, zeroed here) of a 3x3x3 convolution with stride 1 or 2 (see file header).
int tb_conv3d_wgrad_f32(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
                        int Hi, int Wi, int stride, int pad, void* stream) {
  if (!G || !X || !dW || N < 1 || M < 1 || Cc < 1 || Do < 1 || Ho < 1 || Wo < 1 || Di < 1 || Hi < 1 || Wi < 1)
    return TB_ERR_INVALID_ARG;
  if (stride != 1 && stride != 2) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * Cc * 27, st) != hipSuccess) return TB_ERR_HIP;
  const bool small = (Wo % 64 != 0) && ((Wo + 31) / 32 * 32 <= (Wo + 63) / 64 * 64 - 16);
  if (stride == 1)
    return small ? launch<1, 32>(G, X, dW, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, pad, st)
                 : launch<1, 64>(G, X, dW, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, pad, st);
  return small ? launch<2, 32>(G, X, dW, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, pad, st)
               : launch<2, 64>(G, X, dW, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, pad, st);
}
