// conv_wgrad.hip -- 3-D convolution weight gradient (f32, MFMA 16x16x4) for the U-Net train step.
//
// The reference trains MONAI's 3-D U-Net (10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-204)
// and its backward needs dW of every Conv3d / ConvTranspose3d.  MIOpen on gfx950 runs the weight
// gradient of the full- and half-resolution layers (K = N * 120*120*80 = 2.3 M reduction positions,
// only 16 x 16 x 27 outputs) with a naive kernel or a CK GEMM without split-K: ~350 ms each.
// This kernel is a split-K implicit GEMM:
//   dW[m][c][tz][ty][tx] = sum_n sum_{z,y,x} G[n][m][z][y][x] * X[n][c][s z + tz - 1][s y + ty - 1][s x + tx - 1]
// which covers both layer kinds:
//   Conv3d          : G = dY [N][Cout][out],  X = x  [N][Cin][in],   dW = [Cout][Cin][k^3]
//   ConvTranspose3d : G = x  [N][Cin][in],    X = dY [N][Cout][out], dW = [Cin][Cout][k^3]
// (PyTorch's transposed conv places x[q] at s q - p + t, the same index map).
//
// v_mfma_f32_16x16x4_f32: rows = 16 output channels m, K = 4 consecutive x positions, columns =
//   TX = 1: 16 input channels c; the 27 taps (tz,ty,tx) are accumulators split over the 4 waves;
//   TX = 3: (c, tx) pairs of up to 5 channels -- the 3- and 4-channel layers fill 9-12 of the 16
//           columns instead of 3-4 -- and the 9 (tz,ty) taps are the accumulators.
// Work unit ("chunk") = (n, z, YB consecutive output rows, every x): the block stages G[16][YB][Wo]
// and the input rows X[c][tz][S(YB-1)+3][x + halo] in LDS once and runs YB * Wo/4 k-steps of every
// tap over them (each staged input row feeds up to 27 MFMA taps).  Rows are staged whole by one
// wave each (scalar row bounds) as global->LDS DMA, every row of the chunk in flight at once.  At most ~78 KB of
// LDS so two blocks share a CU and one block's staging hides under the other's MFMAs.  Partial sums
// leave each block once, by float atomics into dW (zeroed first).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "texbias.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;
constexpr int LDS_FLOATS = 78 * 1024 / 4;
constexpr int kSlack = 16;  // floats after the carve: the pipelined operand read one k-step past a row

struct WgArgs {
  const float* G;
  const float* X;
  float* dW;
  int M, Cc, Do, Ho, Wo, Di, Hi, Wi;
  int YB, YR, Wo4, XP, PG, PC, ncc, ctiles, nyb, xcols;
  int64_t nchunks;
};

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// lanes copy src[x] -> dst[x], x < n, by 4-B global->LDS DMA pieces (dst wave-uniform)
template <int SEG>
__device__ __forceinline__ void copy_row(const float* src, float* dst, int n, int lane) {
#pragma unroll
  for (int s = 0; s < SEG; ++s) {
    const int x = lane + 64 * s;
    if (x < n) __builtin_amdgcn_global_load_lds((gptr_t)(src + x), (lptr_t)(dst + 64 * s), 4, 0, 0);
  }
}
template <int SEG>
__device__ __forceinline__ void zero_row(float* dst, int n, int lane) {
#pragma unroll
  for (int s = 0; s < SEG; ++s) {
    const int x = lane + 64 * s;
    if (x < n) dst[x] = 0.f;
  }
}

template <int S, int TX, int SEG>
__global__ __launch_bounds__(NT) void k_conv3d_wgrad(WgArgs a) {
  constexpr int NTAP = TX == 1 ? 27 : 9;
  constexpr int TPW = (NTAP + 3) / 4;  // taps per wave (the last wave may have one fewer)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mt = (int)blockIdx.y / a.ctiles, ct = (int)blockIdx.y - mt * a.ctiles;
  const int m0 = mt * 16, c0 = ct * a.ncc;
  const int mv = min(16, a.M - m0), cv = min(a.ncc, a.Cc - c0);
  // the carve holds only this block's mv rows and cv channel planes; lanes of absent rows / columns
  // read row 0 / plane 0 (their MFMA results are never stored)
  float* gs = smem;               // [mv][PG]   row m: YB rows of Wo4 (zero beyond Wo)
  float* xs = smem + mv * a.PG;   // [cv][PC]   plane c: [3 tz][YR rows][XP], col 0 = left halo
  const int nlds = mv * a.PG + cv * a.PC + kSlack;
  for (int i = tid; i < nlds; i += NT) smem[i] = 0.f;   // halos, x >= Wo, absent m / c stay zero
  const int li = lane & 15, lk = lane >> 4;
  int boff;
  if (TX == 1) {
    boff = (li < cv ? li : 0) * a.PC;
  } else {
    const int c = li / 3, tx = li - 3 * c;
    boff = c < cv ? c * a.PC + tx : 0;
  }
  int toff[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + 4 * j < NTAP ? wave + 4 * j : 0;
    toff[j] = TX == 1 ? ((t / 9) * a.YR + (t / 3) % 3) * a.XP + t % 3 : ((t / 3) * a.YR + t % 3) * a.XP;
  }
  f32x4 acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t gsm = (int64_t)a.Do * a.Ho * a.Wo, xsc = (int64_t)a.Di * a.Hi * a.Wi;
  __syncthreads();

  for (int64_t ch = blockIdx.x; ch < a.nchunks; ch += gridDim.x) {
    int64_t r = ch;
    const int yb = (int)(r % a.nyb);
    r /= a.nyb;
    const int z = (int)(r % a.Do);
    const int n = (int)(r / a.Do);
    const int y0 = yb * a.YB;
    // Staging: one wave per row, rows dealt round-robin to the 4 waves; in-range rows go global ->
    // LDS by DMA (global_load_lds, lane-linear 4-B pieces, no registers, all of a wave's rows in
    // flight at once), out-of-range rows (z / y halo) are zero-filled.  The barrier below drains them.
    const float* gb = a.G + ((int64_t)n * a.M + m0) * gsm + (int64_t)z * a.Ho * a.Wo;
    int row = 0;
    for (int m = 0; m < mv; ++m)
      for (int yy = 0; yy < a.YB; ++yy, ++row) {
        if ((row & 3) != wave) continue;
        const int y = y0 + yy;
        float* dst = gs + m * a.PG + yy * a.Wo4;
        if (y < a.Ho) copy_row<SEG>(gb + m * gsm + (int64_t)y * a.Wo, dst, a.Wo, lane);
        else zero_row<SEG>(dst, a.Wo, lane);
      }
    const float* xb0 = a.X + ((int64_t)n * a.Cc + c0) * xsc;
    row = 0;
    for (int c = 0; c < cv; ++c)
      for (int tz = 0; tz < 3; ++tz) {
        const int zi = S * z + tz - 1;
        for (int yr = 0; yr < a.YR; ++yr, ++row) {
          if ((row & 3) != wave) continue;
          const int yi = S * y0 + yr - 1;
          float* dst = xs + c * a.PC + (tz * a.YR + yr) * a.XP + 1;
          if (zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi)
            copy_row<SEG>(xb0 + c * xsc + ((int64_t)zi * a.Hi + yi) * a.Wi, dst, a.xcols, lane);
          else
            zero_row<SEG>(dst, a.xcols, lane);
        }
      }
    __syncthreads();
    // k-steps of 4 x positions: every wave runs TPW taps with no per-tap branch (a wave's taps past
    // NTAP read a valid address and are never stored); the operands of step x0 + 4 are read while
    // the MFMAs of step x0 run (the read past the row end stays inside the carve's slack)
    for (int yy = 0; yy < a.YB; ++yy) {
      const float* ga = gs + (li < mv ? li : 0) * a.PG + yy * a.Wo4 + lk;
      const float* xq = xs + boff + (S * yy) * a.XP + S * lk;
      float av = ga[0];
      float bv[TPW];
#pragma unroll
      for (int j = 0; j < TPW; ++j) bv[j] = xq[toff[j]];
      for (int x0 = 0; x0 < a.Wo4; x0 += 4) {
        const float an = ga[x0 + 4];
        float bn[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j) bn[j] = xq[toff[j] + S * (x0 + 4)];
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j], acc[j], 0, 0, 0);
        av = an;
#pragma unroll
        for (int j = 0; j < TPW; ++j) bv[j] = bn[j];
      }
    }
    __syncthreads();
  }
  // D[row = m][col]: lane holds rows (lane>>4)*4 + rr, column lane & 15
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + 4 * j;
    if (t >= NTAP) continue;
    int c, tap;
    if (TX == 1) {
      c = li;
      tap = t;
      if (c >= cv) continue;
    } else {
      c = li / 3;
      tap = t * 3 + (li - 3 * c);
      if (li >= 3 * cv) continue;
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = lk * 4 + rr;
      if (m < mv) atomicAdd(&a.dW[((int64_t)(m0 + m) * a.Cc + (c0 + c)) * 27 + tap], acc[j][rr]);
    }
  }
}

// Stride 1, at most 5 output and 5 input channels (the top ResidualUnit's 3 -> 3 conv at full
// resolution): the (c, tx) columns above leave 13 of the 16 MFMA rows empty (3 output channels).
// Here the rows are (m, tz) and the chunk is an INPUT plane zi: with z = zi - tz + 1,
//   dW[m][c][tz][ty][tx] += sum_{y,x} G[m][zi - tz + 1][y][x] * X[c][zi][y + ty - 1][x + tx - 1]
// so one staged input plane serves all three tz at once (rows 3 m + tz <= 15, columns 3 c + tx <= 15)
// and only the three ty taps remain accumulators: a third of the MFMAs of the (c, tx) form.  Chunk =
// (n, zi, YB output rows); stage G[m][3 planes][YB rows][Wo4] and X[c][YB + 2 rows][x + halo]; the
// four waves take alternate rows yy and keep all three ty accumulators; partial sums leave by float
// atomics as above.
template <int SEG>
__global__ __launch_bounds__(NT) void k_conv3d_wgrad_mz(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.M, Cc = a.Cc;
  float* gs = smem;               // [3 M][PG]   row (m, tz): YB rows of Wo4 (zero beyond Wo)
  float* xs = smem + 3 * M * a.PG;  // [Cc][PC]  plane c: [YR rows][XP], col 0 = left halo
  const int nlds = 3 * M * a.PG + Cc * a.PC + kSlack;
  for (int i = tid; i < nlds; i += NT) smem[i] = 0.f;
  const int li = lane & 15, lk = lane >> 4;
  const int ar = li < 3 * M ? li : 0;                          // A row (m, tz)
  const int bc = li < 3 * Cc ? li / 3 : 0, btx = li < 3 * Cc ? li - 3 * (li / 3) : 0;
  const int boff = bc * a.PC + btx;
  f32x4 acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t gsm = (int64_t)a.Do * a.Ho * a.Wo, xsc = (int64_t)a.Di * a.Hi * a.Wi;
  __syncthreads();
  for (int64_t ch = blockIdx.x; ch < a.nchunks; ch += gridDim.x) {
    int64_t r = ch;
    const int yb = (int)(r % a.nyb);
    r /= a.nyb;
    const int zi = (int)(r % a.Di);
    const int n = (int)(r / a.Di);
    const int y0 = yb * a.YB;
    int row = 0;
    for (int m = 0; m < M; ++m)
      for (int tz = 0; tz < 3; ++tz) {
        const int z = zi - tz + 1;
        const float* gb = a.G + ((int64_t)n * M + m) * gsm + (int64_t)z * a.Ho * a.Wo;
        for (int yy = 0; yy < a.YB; ++yy, ++row) {
          if ((row & 3) != wave) continue;
          const int y = y0 + yy;
          float* dst = gs + (m * 3 + tz) * a.PG + yy * a.Wo4;
          if (z >= 0 && z < a.Do && y < a.Ho) copy_row<SEG>(gb + (int64_t)y * a.Wo, dst, a.Wo, lane);
          else zero_row<SEG>(dst, a.Wo, lane);
        }
      }
    const float* xb0 = a.X + (int64_t)n * Cc * xsc + (int64_t)zi * a.Hi * a.Wi;
    row = 0;
    for (int c = 0; c < Cc; ++c)
      for (int yr = 0; yr < a.YR; ++yr, ++row) {
        if ((row & 3) != wave) continue;
        const int yi = y0 + yr - 1;
        float* dst = xs + c * a.PC + yr * a.XP + 1;
        if (yi >= 0 && yi < a.Hi) copy_row<SEG>(xb0 + c * xsc + (int64_t)yi * a.Wi, dst, a.xcols, lane);
        else zero_row<SEG>(dst, a.xcols, lane);
      }
    __syncthreads();
    for (int yy = wave; yy < a.YB; yy += 4) {
      const float* ga = gs + ar * a.PG + yy * a.Wo4 + lk;
      const float* xq = xs + boff + yy * a.XP + lk;  // + ty XP for tap ty
      float av = ga[0];
      float bv[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) bv[j] = xq[j * a.XP];
      for (int x0 = 0; x0 < a.Wo4; x0 += 4) {
        const float an = ga[x0 + 4];
        float bn[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) bn[j] = xq[j * a.XP + x0 + 4];
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j], acc[j], 0, 0, 0);
        av = an;
#pragma unroll
        for (int j = 0; j < 3; ++j) bv[j] = bn[j];
      }
    }
    __syncthreads();
  }
  // D[row = (m, tz)][col = (c, tx)]: lane holds rows (lane >> 4) * 4 + rr, column lane & 15.  The
  // four waves' sums meet in LDS first, so a block adds each dW entry once (thousands of blocks'
  // atomics on the same 3 M Cc 27 addresses serialise).
  float* red = smem;  // [4 waves][3 taps][4 rr][64 lanes]
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[((wave * 3 + j) * 4 + rr) * 64 + lane] = acc[j][rr];
  __syncthreads();
  if (wave != 0 || li >= 3 * Cc) return;
  const int c = li / 3, tx = li - 3 * c;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int rw = lk * 4 + rr;
      if (rw >= 3 * M) continue;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[((w * 3 + j) * 4 + rr) * 64 + lane];
      const int m = rw / 3, tz = rw - 3 * m;
      atomicAdd(&a.dW[((int64_t)m * Cc + c) * 27 + tz * 9 + j * 3 + tx], v);
    }
}

int pad_mod32(int v, int rem) {
  while ((v & 31) != rem) ++v;
  return v;
}

template <int S, int TX, int SEG>
int launch(const WgArgs& a, int blocks_y, size_t lds, hipStream_t st) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3d_wgrad<S, TX, SEG>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return TB_ERR_HIP;
  // two blocks per CU over the whole chip (TEXBIAS_WGRAD_BLOCKS overrides, tuning), never more
  // chunks than exist
  static const int target = [] {
    const char* e = std::getenv("TEXBIAS_WGRAD_BLOCKS");
    return e ? std::atoi(e) : 512;
  }();
  int64_t gx = (target + blocks_y - 1) / blocks_y;
  if (gx > a.nchunks) gx = a.nchunks;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((k_conv3d_wgrad<S, TX, SEG>), dim3((unsigned)gx, (unsigned)blocks_y), dim3(NT), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

template <int S, int TX>
int launch_seg(const WgArgs& a, int seg, int by, size_t lds, hipStream_t st) {
  switch (seg) {
    case 1: return launch<S, TX, 1>(a, by, lds, st);
    case 2: return launch<S, TX, 2>(a, by, lds, st);
    case 3: return launch<S, TX, 3>(a, by, lds, st);
    case 4: return launch<S, TX, 4>(a, by, lds, st);
    default: return TB_ERR_UNSUPPORTED_SIZE;
  }
}

// Tiling of one weight-gradient call: TX (taps vs (c, tx) columns), SEG (64-wide row segments a
// wave stages) and YB (output rows per chunk, the largest that fits the LDS budget).
// (m, tz)-row tiling of k_conv3d_wgrad_mz (TX = 9 in the config query): stride 1, M, Cc <= 5
int wg_setup_mz(WgArgs& a, int& seg, int& by, size_t& lds, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
                int Hi, int Wi) {
  a.M = M; a.Cc = Cc; a.Do = Do; a.Ho = Ho; a.Wo = Wo; a.Di = Di; a.Hi = Hi; a.Wi = Wi;
  a.Wo4 = (Wo + 3) / 4 * 4;
  const int xw = a.Wo4 - 1 + 3;                       // staged columns incl. the left halo
  a.XP = xw | 1;
  a.xcols = Wi < a.XP - 1 ? Wi : a.XP - 1;
  seg = (((Wo > a.xcols ? Wo : a.xcols) + 63) / 64);
  if (seg > 4) return TB_ERR_UNSUPPORTED_SIZE;
  a.YB = 0;
  static const int yb_max = [] {  // TEXBIAS_WGRAD_MZ_YB caps the rows per chunk (tuning)
    const char* e = std::getenv("TEXBIAS_WGRAD_MZ_YB");
    return e ? std::atoi(e) : 4;  // 3->3 at 2x240x240x160: YB 8 / 512 blocks 530 us, YB 4 / 1024 blocks 462 us
  }();
  for (int yb : {8, 4, 2, 1}) {
    if ((yb > 1 && yb > Ho) || yb > yb_max) continue;
    const int yr = yb + 2;
    const int pg = pad_mod32(yb * a.Wo4, 2);
    const int pc = pad_mod32(yr * a.XP, 3);
    if (3 * M * pg + Cc * pc + kSlack <= LDS_FLOATS) {
      a.YB = yb; a.YR = yr; a.PG = pg; a.PC = pc;
      break;
    }
  }
  if (!a.YB) return TB_ERR_UNSUPPORTED_SIZE;
  a.nyb = (Ho + a.YB - 1) / a.YB;
  a.nchunks = (int64_t)N * Di * a.nyb;
  const int carve = 3 * M * a.PG + Cc * a.PC + kSlack;
  lds = sizeof(float) * (size_t)(carve > 4 * 3 * 4 * 64 ? carve : 4 * 3 * 4 * 64);  // >= the end's wave sums
  by = 1;
  return TB_OK;
}

template <int SEG>
int launch_mz(const WgArgs& a, size_t lds, hipStream_t st) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3d_wgrad_mz<SEG>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return TB_ERR_HIP;
  static const int target = [] {
    const char* e = std::getenv("TEXBIAS_WGRAD_MZ_BLOCKS");
    return e ? std::atoi(e) : 1024;
  }();
  int64_t gx = target;
  if (gx > a.nchunks) gx = a.nchunks;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(k_conv3d_wgrad_mz<SEG>, dim3((unsigned)gx), dim3(NT), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

bool use_mz(int M, int Cc, int stride) {
  static const bool on = [] {
    const char* e = std::getenv("TEXBIAS_WGRAD_MZ");
    return !(e && e[0] == '0');
  }();
  return on && stride == 1 && M <= 5 && Cc <= 5;
}

int wg_setup(WgArgs& a, int& seg, int& TX, int& by, size_t& lds, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
             int Hi, int Wi, int stride, int pad) {
  if (N < 1 || M < 1 || Cc < 1 || Do < 1 || Ho < 1 || Wo < 1 || Di < 1 || Hi < 1 || Wi < 1) return TB_ERR_INVALID_ARG;
  if ((stride != 1 && stride != 2) || pad != 1) return TB_ERR_INVALID_ARG;
  if (use_mz(M, Cc, stride)) {
    TX = 9;
    return wg_setup_mz(a, seg, by, lds, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi);
  }
  a.M = M; a.Cc = Cc; a.Do = Do; a.Ho = Ho; a.Wo = Wo; a.Di = Di; a.Hi = Hi; a.Wi = Wi;
  TX = Cc <= 5 ? 3 : 1;
  a.ncc = TX == 3 ? 5 : 16;
  a.Wo4 = (Wo + 3) / 4 * 4;
  const int xw = stride * (a.Wo4 - 1) + 3;            // staged columns incl. the left halo
  a.XP = xw | 1;
  a.xcols = Wi < a.XP - 1 ? Wi : a.XP - 1;             // input columns that can be touched
  seg = (((Wo > a.xcols ? Wo : a.xcols) + 63) / 64);
  if (seg > 4) return TB_ERR_UNSUPPORTED_SIZE;
  const int prem = TX == 3 ? 3 : 2;                     // plane pitch mod 32 (bank spread of B reads)
  a.YB = 0;
  static const int yb_max = [] {  // TEXBIAS_WGRAD_YB caps the rows per chunk (tuning)
    const char* e = std::getenv("TEXBIAS_WGRAD_YB");
    return e ? std::atoi(e) : 8;
  }();
  for (int yb : {8, 4, 2, 1}) {
    if ((yb > 1 && yb > Ho) || yb > yb_max) continue;
    const int yr = stride * (yb - 1) + 3;
    const int pg = pad_mod32(yb * a.Wo4, 2);
    const int pc = pad_mod32(3 * yr * a.XP, prem);
    if ((M < 16 ? M : 16) * pg + (Cc < a.ncc ? Cc : a.ncc) * pc + kSlack <= LDS_FLOATS) {
      a.YB = yb; a.YR = yr; a.PG = pg; a.PC = pc;
      break;
    }
  }
  if (!a.YB) return TB_ERR_UNSUPPORTED_SIZE;
  a.nyb = (Ho + a.YB - 1) / a.YB;
  a.nchunks = (int64_t)N * Do * a.nyb;
  const int mtiles = (M + 15) / 16;
  a.ctiles = (Cc + a.ncc - 1) / a.ncc;
  lds = sizeof(float) * (size_t)((M < 16 ? M : 16) * a.PG + (Cc < a.ncc ? Cc : a.ncc) * a.PC + kSlack);
  by = mtiles * a.ctiles;
  return TB_OK;
}

}  // namespace

// dW (M x Cc x 27, zeroed here) of a 3x3x3 convolution with stride 1 or 2, padding 1 (file header).
int tb_conv3d_wgrad_f32(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
                        int Hi, int Wi, int stride, int pad, void* stream) {
  if (!G || !X || !dW) return TB_ERR_INVALID_ARG;
  WgArgs a{};
  int seg = 0, TX = 0, by = 0;
  size_t lds = 0;
  const int rc = wg_setup(a, seg, TX, by, lds, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad);
  if (rc != TB_OK) return rc;
  a.G = G; a.X = X; a.dW = dW;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * Cc * 27, st) != hipSuccess) return TB_ERR_HIP;
  if (TX == 9) {
    switch (seg) {
      case 1: return launch_mz<1>(a, lds, st);
      case 2: return launch_mz<2>(a, lds, st);
      case 3: return launch_mz<3>(a, lds, st);
      case 4: return launch_mz<4>(a, lds, st);
      default: return TB_ERR_UNSUPPORTED_SIZE;
    }
  }
  if (stride == 1) return TX == 1 ? launch_seg<1, 1>(a, seg, by, lds, st) : launch_seg<1, 3>(a, seg, by, lds, st);
  return TX == 1 ? launch_seg<2, 1>(a, seg, by, lds, st) : launch_seg<2, 3>(a, seg, by, lds, st);
}

// The tiling tb_conv3d_wgrad_f32 would choose (no launch): cfg = {SEG, TX, YB, chunks, LDS bytes}.
int tb_conv3d_wgrad_config(int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi, int Wi, int stride, int pad,
                           int64_t* cfg) {
  if (!cfg) return TB_ERR_INVALID_ARG;
  WgArgs a{};
  int seg = 0, TX = 0, by = 0;
  size_t lds = 0;
  const int rc = wg_setup(a, seg, TX, by, lds, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad);
  if (rc != TB_OK) return rc;
  cfg[0] = seg; cfg[1] = TX; cfg[2] = a.YB; cfg[3] = a.nchunks; cfg[4] = (int64_t)lds;
  return TB_OK;
}
