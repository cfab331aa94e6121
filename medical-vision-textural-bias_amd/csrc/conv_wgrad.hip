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


// ---------------------------------------------------------------------------------------------
// Stride 1, 16-channel tiles: the block MARCHES along the input planes zi of its (n, YB-row block,
// z segment).  With z = zi - tz + 1,
//   dW[m][c][tz][ty][tx] += sum_{y,x} G[m][zi - tz + 1][y][x] * X[c][zi][y + ty - 1][x + tx - 1]
// so one staged input plane (X slab: 16 c x (YB + 2) rows + x halo) meets the three G planes
// zi + 1, zi, zi - 1 kept in a 4-slot ring: every z step stages ONE new X slab and ONE new G slab
// (the im2col re-staging of the chunked kernel was 6x the input per output plane).  Each k-step of 4
// positions reads 3 A fragments (the tz planes) and 9 B fragments (the (ty, tx) shifts) for 27 MFMAs
// (16x16x4 f32: rows m, columns c) into 27 accumulators per wave; the waves split the positions and
// meet in LDS at the end, one float atomic per dW entry per block.  The next plane's slabs are loaded
// into registers while the current plane's MFMAs run (one barrier per z step).
constexpr size_t ZM_RED_BYTES = (size_t)27 * 2 * 4 * 64 * 4;  // k_conv3d_wgrad_zm end reduction

struct ZmArgs {
  const float* G;
  const float* X;
  float* dW;
  float* part;  // non-null: per-workgroup partial tiles [tile][block][16 m][16 c][27] instead of atomics
  int N, M, Cc, D, H, W;       // G and X both [N][.][D][H][W] (stride 1, padding 1)
  int YB, nyb, ZS, zlen;       // rows per block, row blocks, z segments, planes per segment
  int MS, RX, PX, W4;          // LDS pitches (floats): G channel, X channel, X row; k-step row length
  int mtiles, ctiles;
};

// NW waves share the block's ring (8: two per SIMD at one block per CU): the row's k-steps are split
// over NW / YB waves; at the end the waves hand their sums down two at a time through a 2-wave LDS
// image (55.3 KB, inside the ring's allocation), then one atomic per dW entry per block.
template <int YB, int WV, int NW>  // WV: most float4 per row (W <= 4 WV)
__global__ __launch_bounds__(64 * NW) void k_conv3d_wgrad_zm(ZmArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int NXR = YB + 2;  // staged X rows
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H, D = a.D, W4 = a.W4;
  const int GS = 16 * a.MS, XS = 16 * a.RX;  // slab sizes
  float* gsl = smem;                        // [4 slots][16 m][MS]: row yy at yy * W4, zero past W
  float* xsl = smem + 4 * GS;               // [2 slots][16 c][RX]: row r at r * PX, x at col x + 2
  // block -> (tile, n, row block, z segment)
  const int tile = (int)blockIdx.y, mt = tile / a.ctiles, ct = tile - mt * a.ctiles;
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int m0 = 16 * mt, c0 = 16 * ct;
  const int mv = min(16, a.M - m0), cv = min(16, a.Cc - c0);
  const int y0 = yb * YB;
  const int z0 = zs * a.zlen, z1 = min(D, z0 + a.zlen);
  for (int i = tid; i < 4 * GS + 2 * XS; i += NT) smem[i] = 0.f;  // halos, pads, absent rows stay 0
  const int64_t plane = (int64_t)H * W;
  const float* Gb = a.G + ((int64_t)n * a.M + m0) * D * plane;
  const float* Xb = a.X + ((int64_t)n * a.Cc + c0) * D * plane;
  // staging items, fixed per thread for the whole march: global offset within a plane (-1: none)
  // and LDS offset within a slab -- X (c, r, q) with row y0 - 1 + r in range, G (m, yy, q)
  const int W4v = W >> 2;
  constexpr int NXL = (16 * NXR * WV + NT - 1) / NT, NGL = (16 * YB * WV + NT - 1) / NT;
  int xg[NXL], xl[NXL], gg[NGL], gl[NGL];
#pragma unroll
  for (int j = 0; j < NXL; ++j) {
    const int i = tid + NT * j;
    const int q = i % W4v, t = i / W4v, r = t % NXR, c = t / NXR;
    const int y = y0 - 1 + r;
    const bool ok = c < cv && y >= 0 && y < H;
    xg[j] = ok ? (int)(((int64_t)c * D) * plane / 4 + (y * W + 4 * q) / 4) : -1;  // in float4 of the plane-0 base
    xl[j] = c * a.RX + r * a.PX + 2 + 4 * q;
  }
#pragma unroll
  for (int j = 0; j < NGL; ++j) {
    const int i = tid + NT * j;
    const int q = i % W4v, t = i / W4v, yy = t % YB, m = t / YB;
    const int y = y0 + yy;
    const bool ok = m < mv && y < H;
    gg[j] = ok ? (int)(((int64_t)m * D) * plane / 4 + (y * W + 4 * q) / 4) : -1;
    gl[j] = m * a.MS + yy * W4 + 4 * q;
  }
  float4 rx[NXL], rg[NGL];
  const int64_t plane4 = plane / 4;
  // (zero-selects at the LDS store, not at the load: a select right after a load makes the wave wait
  // for it there, and the next plane's loads would not overlap this plane's MFMAs)
  auto load_x = [&](int zi) {
    const float4* src = reinterpret_cast<const float4*>(Xb) + (int64_t)zi * plane4;
#pragma unroll
    for (int j = 0; j < NXL; ++j) rx[j] = src[xg[j] < 0 ? 0 : xg[j]];
  };
  auto store_x = [&](int slot) {
    float* d = xsl + slot * XS;
#pragma unroll
    for (int j = 0; j < NXL; ++j)
      if (xg[j] >= 0) {
        float2* p = reinterpret_cast<float2*>(d + xl[j]);
        p[0] = make_float2(rx[j].x, rx[j].y);
        p[1] = make_float2(rx[j].z, rx[j].w);
      }
  };
  bool gin = false;             // the G plane in rg lies inside [0, D) (else stored as zeros)
  auto load_g = [&](int pz) {  // G plane pz (zero outside [0, D))
    gin = pz >= 0 && pz < D;
    const float4* src = reinterpret_cast<const float4*>(Gb) + (int64_t)(gin ? pz : 0) * plane4;
#pragma unroll
    for (int j = 0; j < NGL; ++j) rg[j] = src[gg[j] < 0 ? 0 : gg[j]];
  };
  auto store_g = [&](int slot) {
    float* d = gsl + slot * GS;
#pragma unroll
    for (int j = 0; j < NGL; ++j)
      if (gg[j] >= 0) {
        const float4 v = gin ? rg[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        float2* p = reinterpret_cast<float2*>(d + gl[j]);
        p[0] = make_float2(v.x, v.y);
        p[1] = make_float2(v.z, v.w);
      }
  };
  __syncthreads();  // the zero fill is done before any slab store
  // prologue: G planes z0 - 1 and z0 into their ring slots, then X[z0] and G[z0 + 1] in registers
  load_g(z0 - 1);
  store_g((z0 + 3) & 3);
  load_g(z0);
  store_g(z0 & 3);
  load_x(z0);
  load_g(z0 + 1);

  const int li = lane & 15, lk = lane >> 4;
  const int aoff = li * a.MS + lk;                 // A: G[m = li][yy][x0 + lk]
  const int boff = li * a.RX + lk + 1;             // B: X[c = li][yy + ty][x0 + lk + tx - 1] at col + 2
  const int kpr = W4 >> 2;                         // k-steps per row
  f32x4 acc[27];
#pragma unroll
  for (int j = 0; j < 27; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int zi = z0; zi < z1; ++zi) {
    store_x(zi & 1);
    store_g((zi + 1) & 3);
    __syncthreads();  // slabs of this step visible; every wave is past the step that last read these slots
    // next step's slabs fly during this step's MFMAs -- unconditionally (after the last step a clamped,
    // never-stored plane): a conditional load leaves a register merge at the loop edge whose copies wait
    // for the loads before the MFMAs
    load_x(zi + 1 < D ? zi + 1 : zi);
    load_g(zi + 2);
    const float* g0 = gsl + ((zi + 1) & 3) * GS + aoff;  // tz = 0: plane zi + 1
    const float* g1 = gsl + (zi & 3) * GS + aoff;        // tz = 1: plane zi
    const float* g2 = gsl + ((zi + 3) & 3) * GS + aoff;  // tz = 2: plane zi - 1
    const float* xb = xsl + (zi & 1) * XS + boff;
    // this wave's k-steps: row yy = wave % YB, x0 over part wave / YB of the row (4 / YB parts);
    // the next k-step's 12 operands are read under the current one's 27 MFMAs (2x unrolled, clamped)
    const int yy = wave % YB, np = NW / YB, part = wave / YB;
    const int kb = (kpr * part) / np, ke = (kpr * (part + 1)) / np;
    auto ld = [&](int k, float (&av)[3], float (&bv)[9]) {
      const int kk = k < ke ? k : ke - 1;
      const int ga = yy * W4 + 4 * kk, xa = yy * a.PX + 4 * kk;
      av[0] = g0[ga];
      av[1] = g1[ga];
      av[2] = g2[ga];
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) bv[ty * 3 + tx] = xb[xa + ty * a.PX + tx];
    };
    auto mm = [&](const float (&av)[3], const float (&bv)[9]) {
#pragma unroll
      for (int tz = 0; tz < 3; ++tz)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[tz * 9 + t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[tz], bv[t], acc[tz * 9 + t], 0, 0, 0);
    };
    if (kb < ke) {
      float a0[3], b0[9], a1[3], b1[9];
      ld(kb, a0, b0);
      int k = kb;
      for (; k + 1 < ke; k += 2) {
        ld(k + 1, a1, b1);
        mm(a0, b0);
        ld(k + 2, a0, b0);
        mm(a1, b1);
      }
      if (k < ke) mm(a0, b0);
    }
  }
  // the waves' sums meet in LDS two at a time (the ring is free after the first barrier)
  float* red = smem;  // [27][2 waves][4 rr][64 lanes]
#pragma unroll
  for (int hw = NW - 2; hw >= 2; hw -= 2) {  // waves hw, hw + 1 hand their sums to hw - 2, hw - 1
    __syncthreads();
    if (wave >= hw && wave < hw + 2) {
#pragma unroll
      for (int j = 0; j < 27; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) red[((j * 2 + wave - hw) * 4 + rr) * 64 + lane] = acc[j][rr];
    }
    __syncthreads();
    if (wave >= hw - 2 && wave < hw) {
#pragma unroll
      for (int j = 0; j < 27; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[j][rr] += red[((j * 2 + wave - hw + 2) * 4 + rr) * 64 + lane];
    }
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int j = 0; j < 27; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[((j * 2 + wave) * 4 + rr) * 64 + lane] = acc[j][rr];
  }
  __syncthreads();
  float* pt = a.part ? a.part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (16 * 16 * 27) : nullptr;
  for (int e = tid; e < 27 * 4 * 64; e += NT) {  // e = (j, rr, lane)
    const int ln = e & 63, rr = (e >> 6) & 3, j = e >> 8;
    const int m = (ln >> 4) * 4 + rr, c = ln & 15;
    const float v = red[((j * 2 + 0) * 4 + rr) * 64 + ln] + red[((j * 2 + 1) * 4 + rr) * 64 + ln];
    if (pt) {
      pt[(m * 16 + c) * 27 + j] = v;  // the whole tile (zeros past mv, cv: those G / X rows were staged as 0)
    } else if (m < mv && c < cv) {
      atomicAdd(&a.dW[((int64_t)(m0 + m) * a.Cc + (c0 + c)) * 27 + j], v);
    }
  }
}

// dW from per-workgroup partial tiles part[tile][nblk][TM m][TC c][27], summed in block order: 64 entries x
// 16 block groups per 1024-thread workgroup (each thread ~nblk / 16 independent loads in flight), the groups
// met in LDS.  grid (ceil(TM TC 27 / 64), tiles); tile -> (mt, ct) = (tile / ctiles, tile % ctiles).
__global__ __launch_bounds__(1024) void k_wgrad_reduce(const float* __restrict__ part, float* __restrict__ dW, int nblk,
                                                       int TM, int TC, int ctiles, int M, int Cc) {
  __shared__ float red[16][64];
  const int tid = (int)threadIdx.x, el = tid & 63, bg = tid >> 6;
  const int TE = TM * TC * 27, tile = (int)blockIdx.y;
  const int e = (int)blockIdx.x * 64 + el;
  const float* src = part + (int64_t)tile * nblk * TE + (e < TE ? e : 0);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = bg;
  for (; b + 48 < nblk; b += 64) {
    s0 += src[(int64_t)b * TE];
    s1 += src[(int64_t)(b + 16) * TE];
    s2 += src[(int64_t)(b + 32) * TE];
    s3 += src[(int64_t)(b + 48) * TE];
  }
  for (; b < nblk; b += 16) s0 += src[(int64_t)b * TE];
  red[bg][el] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (bg == 0 && e < TE) {
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) v += red[g][el];
    const int mt = tile / ctiles, ct = tile - mt * ctiles;
    const int m = e / (TC * 27), r = e - m * (TC * 27), c = r / 27, j = r - c * 27;
    if (mt * TM + m < M && ct * TC + c < Cc) dW[((int64_t)(mt * TM + m) * Cc + ct * TC + c) * 27 + j] = v;
  }
}


// Stride 2, >= 8 input channels: the block marches along the OUTPUT planes z of its (n, output row y,
// z segment) and keeps the input planes 2z - 1, 2z, 2z + 1 (three rows 2y - 1 .. 2y + 1 each) in a
// 5-slot ring -- consecutive planes share one, so a step stages two new input slabs and one G row per
// m -- for 32 output channels (two 16-row m-tiles) at once.  Waves: (m-tile = wave & 1, every other
// k-step); 27 tap accumulators each, 1 A + 27 B reads per 27 MFMAs (16x16x4 f32, rows m, columns c);
// partner waves of one m-tile meet in LDS at the end, one float atomic per dW entry per block.
struct Zm2Args {
  const float* G;
  const float* X;
  float* dW;
  float* part;  // non-null: per-workgroup partial tiles (k_wgrad_reduce) instead of atomics
  int N, M, Cc, Do, Ho, Wo, Di, Hi, Wi;
  int ZS, zlen, YB, nyb;
  int MS, RX, PX;
  int mtiles, ctiles;  // m-tiles of 32 (pairs), c-tiles of 16
};

// NW = 8 waves (two per SIMD at one block per CU): m-tile = wave & 1, k-step parity = wave >> 1 of NW / 2
template <int YB, int WV, int NW>  // output rows per block, Wo <= 4 WV
__global__ __launch_bounds__(64 * NW) void k_conv3d_wgrad_zm2(Zm2Args a) {
  constexpr int NT = 64 * NW, P = NW / 2;
  constexpr int NXR = 2 * YB + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Wo = a.Wo, Ho = a.Ho, Do = a.Do, Hi = a.Hi, Wi = a.Wi, Di = a.Di;
  const int GS = 32 * a.MS, XS = 16 * a.RX;
  float* gsl = smem;             // [2 slots][32 m][MS]: row yy at yy * Wo
  float* xsl = smem + 2 * GS;    // [5 slots][16 c][RX]: row r (input row 2 y0 - 1 + r) at r * PX, col x + 2
  const int tile = (int)blockIdx.y, mt = tile / a.ctiles, ct = tile - mt * a.ctiles;
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int y0 = yb * YB;
  const int m0 = 32 * mt, c0 = 16 * ct;
  const int mv = min(32, a.M - m0), cv = min(16, a.Cc - c0);
  const int z0 = zs * a.zlen, z1 = min(Do, z0 + a.zlen);
  for (int i = tid; i < 2 * GS + 5 * XS; i += NT) smem[i] = 0.f;
  const int64_t iplane = (int64_t)Hi * Wi, oplane = (int64_t)Ho * Wo;
  const float* Gb = a.G + ((int64_t)n * a.M + m0) * Do * oplane;
  const float* Xb = a.X + ((int64_t)n * a.Cc + c0) * Di * iplane;
  const int Wi4 = Wi >> 2, Wo4 = Wo >> 2;
  constexpr int NXL = (16 * NXR * 2 * WV + NT - 1) / NT, NGL = (32 * YB * WV + NT - 1) / NT;
  int xg[NXL], xl[NXL], gg[NGL], gl[NGL];
#pragma unroll
  for (int j = 0; j < NXL; ++j) {  // (c, r, q): input row 2 y0 - 1 + r
    const int i = tid + NT * j;
    const int q = i % Wi4, t = i / Wi4, r = t % NXR, c = t / NXR;
    const int yi = 2 * y0 - 1 + r;
    const bool ok = c < cv && yi >= 0 && yi < Hi;
    xg[j] = ok ? (int)(((int64_t)c * Di) * iplane / 4 + (yi * Wi + 4 * q) / 4) : -1;
    xl[j] = c * a.RX + r * a.PX + 2 + 4 * q;
  }
#pragma unroll
  for (int j = 0; j < NGL; ++j) {  // (m, yy, q): output row y0 + yy
    const int i = tid + NT * j;
    const int q = i % Wo4, t = i / Wo4, yy = t % YB, m = t / YB;
    const bool ok = m < mv && y0 + yy < Ho;
    gg[j] = ok ? (int)(((int64_t)m * Do) * oplane / 4 + ((y0 + yy) * Wo + 4 * q) / 4) : -1;
    gl[j] = m * a.MS + yy * Wo + 4 * q;
  }
  const int64_t iplane4 = iplane / 4, oplane4 = oplane / 4;
  float4 rx0[NXL], rx1[NXL], rg[NGL];
  auto load_x = [&](int zi, float4 (&rx)[NXL]) {  // input plane zi (zero outside [0, Di), at the store)
    const bool in = zi >= 0 && zi < Di;
    const float4* src = reinterpret_cast<const float4*>(Xb) + (int64_t)(in ? zi : 0) * iplane4;
#pragma unroll
    for (int j = 0; j < NXL; ++j) rx[j] = src[xg[j] < 0 ? 0 : xg[j]];
  };
  auto store_x = [&](int zi, const float4 (&rx)[NXL]) {
    float* d = xsl + ((zi + 5) % 5) * XS;
    const bool in = zi >= 0 && zi < Di;
#pragma unroll
    for (int j = 0; j < NXL; ++j)
      if (xg[j] >= 0) {
        const float4 v = in ? rx[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        float2* p = reinterpret_cast<float2*>(d + xl[j]);
        p[0] = make_float2(v.x, v.y);
        p[1] = make_float2(v.z, v.w);
      }
  };
  auto load_g = [&](int z) {
#pragma unroll
    for (int j = 0; j < NGL; ++j) {
      rg[j] = (reinterpret_cast<const float4*>(Gb) + (int64_t)z * oplane4)[gg[j] < 0 ? 0 : gg[j]];
    }
  };
  auto store_g = [&](int z) {
    float* d = gsl + (z & 1) * GS;
#pragma unroll
    for (int j = 0; j < NGL; ++j)
      if (gg[j] >= 0) {
        float2* p = reinterpret_cast<float2*>(d + gl[j]);
        p[0] = make_float2(rg[j].x, rg[j].y);
        p[1] = make_float2(rg[j].z, rg[j].w);
      }
  };
  __syncthreads();  // zero fill before the first slab store
  // prologue: plane 2 z0 - 1 into its slot; planes 2 z0, 2 z0 + 1 and G[z0] in registers
  load_x(2 * z0 - 1, rx0);
  store_x(2 * z0 - 1, rx0);
  load_x(2 * z0, rx0);
  load_x(2 * z0 + 1, rx1);
  load_g(z0);

  const int li = lane & 15, lk = lane >> 4;
  const int mtl = wave & 1, par = wave >> 1;       // this wave's 16-row m-tile and k-step parity
  const int aoff = (16 * mtl + li) * a.MS + lk;    // A: G[m][x0 + lk]
  const int boff = li * a.RX + 2 * lk + 1;         // B: X[c][row][2 (x0 + lk) + tx - 1] at col + 2
  f32x4 acc[27];
#pragma unroll
  for (int j = 0; j < 27; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int z = z0; z < z1; ++z) {
    store_x(2 * z, rx0);
    store_x(2 * z + 1, rx1);
    store_g(z);
    __syncthreads();
    load_x(2 * z + 2, rx0);  // unconditionally (see k_conv3d_wgrad_zm)
    load_x(2 * z + 3, rx1);
    load_g(z + 1 < z1 ? z + 1 : z);
    const float* ga = gsl + (z & 1) * GS + aoff;
    const float* xp[3] = {xsl + ((2 * z - 1 + 5) % 5) * XS + boff, xsl + ((2 * z) % 5) * XS + boff,
                          xsl + ((2 * z + 1) % 5) * XS + boff};
    // k-steps (yy, x0) of this wave's parity: the next one's 28 operands read under the current
    // one's 27 MFMAs (2x unrolled, clamped)
    const int nk = YB * Wo4;
    auto ld = [&](int k, float& av, float (&bv)[27]) {
      const int kk = k < nk ? k : nk - 1;
      const int yy = YB == 1 ? 0 : (kk >= Wo4 ? 1 : 0), x0 = 4 * (kk - yy * Wo4);
      av = ga[yy * Wo + x0];
#pragma unroll
      for (int tz = 0; tz < 3; ++tz)
#pragma unroll
        for (int ty = 0; ty < 3; ++ty)
#pragma unroll
          for (int tx = 0; tx < 3; ++tx) bv[tz * 9 + ty * 3 + tx] = xp[tz][(2 * yy + ty) * a.PX + 2 * x0 + tx];
    };
    auto mm = [&](float av, const float (&bv)[27]) {
#pragma unroll
      for (int t = 0; t < 27; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[t], acc[t], 0, 0, 0);
    };
    if (par < nk) {
      float a0, a1, b0[27], b1[27];
      ld(par, a0, b0);
      int k = par;
      for (; k + P < nk; k += 2 * P) {
        ld(k + P, a1, b1);
        mm(a0, b0);
        ld(k + 2 * P, a0, b0);
        mm(a1, b1);
      }
      if (k < nk) mm(a0, b0);
    }
  }
  // partner waves (same m-tile, other parities) hand their sums down to parity 0 one parity at a time
  // through LDS; parity 0 stores
  float* red = smem;  // [2 m-tiles][27][4 rr][64 lanes]
#pragma unroll
  for (int src = P - 1; src >= 1; --src) {
    __syncthreads();
    if (par == src) {
#pragma unroll
      for (int j = 0; j < 27; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) red[((mtl * 27 + j) * 4 + rr) * 64 + lane] = acc[j][rr];
    }
    __syncthreads();
    if (par == 0) {
#pragma unroll
      for (int j = 0; j < 27; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[j][rr] += red[((mtl * 27 + j) * 4 + rr) * 64 + lane];
    }
  }
  if (par == 0) {
    const int c = li;
    float* pt = a.part ? a.part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (32 * 16 * 27) : nullptr;
#pragma unroll
    for (int j = 0; j < 27; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = 16 * mtl + lk * 4 + rr;
        if (pt) pt[(m * 16 + c) * 27 + j] = acc[j][rr];  // the whole [32][16][27] tile (zeros past mv, cv)
        else if (m < mv && c < cv) atomicAdd(&a.dW[((int64_t)(m0 + m) * a.Cc + (c0 + c)) * 27 + j], acc[j][rr]);
      }
  }
}


// Stride 2, few (<= 5) input channels (the full-resolution first conv 4 -> 16, its residual, and the
// top transposed conv 32 -> 3 whose X is the 3-channel output gradient): output-plane march as
// k_conv3d_wgrad_zm2, YB output rows per block, and the MFMA columns are (c, tx) pairs (3 C <= 15 of 16)
// with the 9 (tz, ty) taps as accumulators per m-tile -- 1 A + 9 B reads per 9 MFMAs.  These layers
// are HBM-bound (4 B of input per 9 MACs): every input row is staged once per row block.
struct Zf2Args {
  const float* G;
  const float* X;
  float* dW;
  float* part;  // non-null: per-workgroup partial tiles (k_wgrad_reduce) instead of atomics
  int N, M, Cc, Do, Ho, Wo, Di, Hi, Wi;
  int YB, nyb, ZS, zlen;
  int MS, RX, PX;
  int mtiles;  // blocks of MT m-tiles
};

// NW = 8 waves (two per SIMD at one block per CU; the loads of twice as many waves in flight)
template <int YB, int MT, int WV, int NW>  // rows per block, 16-row m-tiles per block, Wo <= 4 WV
__global__ __launch_bounds__(64 * NW) void k_conv3d_wgrad_zf2(Zf2Args a) {
  constexpr int NT = 64 * NW;
  constexpr int NXR = 2 * YB + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Wo = a.Wo, Ho = a.Ho, Do = a.Do, Hi = a.Hi, Wi = a.Wi, Di = a.Di, Cc = a.Cc;
  const int GS = 16 * MT * a.MS, XS = Cc * a.RX;
  float* gsl = smem;             // [2 slots][16 MT m][MS]: row yy at yy * Wo
  float* xsl = smem + 2 * GS;    // [5 slots][Cc][RX]: row r (input row 2 y0 - 1 + r) at r * PX, col x + 2
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int mt = (int)blockIdx.y;
  const int m0 = 16 * MT * mt, mv = min(16 * MT, a.M - m0);
  const int y0 = yb * YB;
  const int z0 = zs * a.zlen, z1 = min(Do, z0 + a.zlen);
  for (int i = tid; i < 2 * GS + 5 * XS; i += NT) smem[i] = 0.f;
  const int64_t iplane = (int64_t)Hi * Wi, oplane = (int64_t)Ho * Wo;
  const float* Gb = a.G + ((int64_t)n * a.M + m0) * Do * oplane;
  const float* Xb = a.X + (int64_t)n * Cc * Di * iplane;
  const int Wi4 = Wi >> 2, Wo4 = Wo >> 2;
  constexpr int NXL = (5 * NXR * 2 * WV + NT - 1) / NT, NGL = (16 * MT * YB * WV + NT - 1) / NT;
  int xg[NXL], xl[NXL], gg[NGL], gl[NGL];
#pragma unroll
  for (int j = 0; j < NXL; ++j) {  // (c, r, q)
    const int i = tid + NT * j;
    const int q = i % Wi4, t = i / Wi4, r = t % NXR, c = t / NXR;
    const int yi = 2 * y0 - 1 + r;
    const bool ok = c < Cc && yi >= 0 && yi < Hi;
    xg[j] = ok ? (int)(((int64_t)c * Di) * iplane / 4 + (yi * Wi + 4 * q) / 4) : -1;
    xl[j] = c * a.RX + r * a.PX + 2 + 4 * q;
  }
#pragma unroll
  for (int j = 0; j < NGL; ++j) {  // (m, yy, q)
    const int i = tid + NT * j;
    const int q = i % Wo4, t = i / Wo4, yy = t % YB, m = t / YB;
    const int y = y0 + yy;
    const bool ok = m < mv && y < Ho;
    gg[j] = ok ? (int)(((int64_t)m * Do) * oplane / 4 + (y * Wo + 4 * q) / 4) : -1;
    gl[j] = m * a.MS + yy * Wo + 4 * q;
  }
  const int64_t iplane4 = iplane / 4, oplane4 = oplane / 4;
  float4 rx0[NXL], rx1[NXL], rg[NGL];
  auto load_x = [&](int zi, float4 (&rx)[NXL]) {  // (zero outside [0, Di) at the store)
    const bool in = zi >= 0 && zi < Di;
    const float4* src = reinterpret_cast<const float4*>(Xb) + (int64_t)(in ? zi : 0) * iplane4;
#pragma unroll
    for (int j = 0; j < NXL; ++j) rx[j] = src[xg[j] < 0 ? 0 : xg[j]];
  };
  auto store_x = [&](int zi, const float4 (&rx)[NXL]) {
    float* d = xsl + ((zi + 5) % 5) * XS;
    const bool in = zi >= 0 && zi < Di;
#pragma unroll
    for (int j = 0; j < NXL; ++j)
      if (xg[j] >= 0) {
        const float4 v = in ? rx[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        float2* p = reinterpret_cast<float2*>(d + xl[j]);
        p[0] = make_float2(v.x, v.y);
        p[1] = make_float2(v.z, v.w);
      }
  };
  auto load_g = [&](int z) {
#pragma unroll
    for (int j = 0; j < NGL; ++j) {
      rg[j] = (reinterpret_cast<const float4*>(Gb) + (int64_t)z * oplane4)[gg[j] < 0 ? 0 : gg[j]];
    }
  };
  auto store_g = [&](int z) {
    float* d = gsl + (z & 1) * GS;
#pragma unroll
    for (int j = 0; j < NGL; ++j)
      if (gg[j] >= 0) {
        float2* p = reinterpret_cast<float2*>(d + gl[j]);
        p[0] = make_float2(rg[j].x, rg[j].y);
        p[1] = make_float2(rg[j].z, rg[j].w);
      }
  };
  __syncthreads();
  load_x(2 * z0 - 1, rx0);
  store_x(2 * z0 - 1, rx0);
  load_x(2 * z0, rx0);
  load_x(2 * z0 + 1, rx1);
  load_g(z0);

  const int li = lane & 15, lk = lane >> 4;
  const int bc = li < 3 * Cc ? li / 3 : 0, btx = li < 3 * Cc ? li - 3 * (li / 3) : 0;
  const int boff = bc * a.RX + btx + 2 * lk + 1;  // B: X[c][row][2 (x0 + lk) + tx - 1] at col + 2
  f32x4 acc[MT][9];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int z = z0; z < z1; ++z) {
    store_x(2 * z, rx0);
    store_x(2 * z + 1, rx1);
    store_g(z);
    __syncthreads();
    load_x(2 * z + 2, rx0);  // unconditionally (see k_conv3d_wgrad_zm)
    load_x(2 * z + 3, rx1);
    load_g(z + 1 < z1 ? z + 1 : z);
    const float* ga = gsl + (z & 1) * GS + li * a.MS + lk;
    const float* xp[3] = {xsl + ((2 * z - 1 + 5) % 5) * XS + boff, xsl + ((2 * z) % 5) * XS + boff,
                          xsl + ((2 * z + 1) % 5) * XS + boff};
    // this wave's k-steps: rows yy = wave, wave + NW, ... (YB >= NW), else x parts of row wave % YB;
    // the next k-step's operands are read under the current one's MFMAs (2x unrolled, clamped)
    const int np = YB >= NW ? 1 : NW / YB, yy0 = YB >= NW ? wave : wave % YB, part = YB >= NW ? 0 : wave / YB;
    const int kb = (Wo4 * part) / np, ke = (Wo4 * (part + 1)) / np;
    auto ld = [&](int yy, int k, float (&av)[MT], float (&bv)[9]) {
      const int x0 = 4 * (k < ke ? k : ke - 1);
#pragma unroll
      for (int t = 0; t < MT; ++t) av[t] = ga[t * 16 * a.MS + yy * Wo + x0];
#pragma unroll
      for (int tz = 0; tz < 3; ++tz)
#pragma unroll
        for (int ty = 0; ty < 3; ++ty) bv[tz * 3 + ty] = xp[tz][(2 * yy + ty) * a.PX + 2 * x0];
    };
    auto mm = [&](const float (&av)[MT], const float (&bv)[9]) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < 9; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bv[j], acc[t][j], 0, 0, 0);
    };
    for (int yy = yy0; yy < YB; yy += NW) {
      if (kb >= ke) break;
      float a0[MT], a1[MT], b0[9], b1[9];
      ld(yy, kb, a0, b0);
      int k = kb;
      for (; k + 1 < ke; k += 2) {
        ld(yy, k + 1, a1, b1);
        mm(a0, b0);
        ld(yy, k + 2, a0, b0);
        mm(a1, b1);
      }
      if (k < ke) mm(a0, b0);
    }
  }
  // the waves' sums meet in LDS, one atomic per entry
  __syncthreads();
  float* red = smem;  // [MT][9][NW waves][4 rr][64]
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[(((t * 9 + j) * NW + wave) * 4 + rr) * 64 + lane] = acc[t][j][rr];
  __syncthreads();
  float* pt = a.part ? a.part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (16 * MT * Cc * 27) : nullptr;
  for (int e = tid; e < MT * 9 * 4 * 64; e += NT) {  // e = ((t, j), rr, lane)
    const int ln = e & 63, rr = (e >> 6) & 3, tj = e >> 8, t = tj / 9, j = tj - 9 * t;
    const int m = 16 * t + (ln >> 4) * 4 + rr, col = ln & 15;
    if ((!pt && m >= mv) || col >= 3 * Cc) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[((tj * NW + w) * 4 + rr) * 64 + ln];
    const int c = col / 3, tx = col - 3 * c;
    if (pt) pt[(m * Cc + c) * 27 + j * 3 + tx] = v;  // the whole [16 MT][Cc][27] tile (zeros past mv)
    else atomicAdd(&a.dW[((int64_t)(m0 + m) * Cc + c) * 27 + j * 3 + tx], v);  // j = (tz, ty)
  }
}

// Stride 1, few channels (9 M <= 32, 3 Cc <= 16: the 3->3 full-resolution layer).  MFMA rows are
// (m, tz, ty) -- 27 of two 16-row tiles at M = 3 -- and columns (c, tx), so one k-step of 4 output
// columns px of input row qy (plane qz) is 2 MFMAs (16x16x4 f32) reading 2 A values and 1 B value
// per lane: A[(m, tz, ty)][px] = G[m][qz - tz + 1][qy - ty + 1][px], B[px][(c, tx)] =
// X[c][qz][qy][px + tx - 1].  The block marches its (n, input row block, z segment) along qz: one
// X plane (YB rows) and one G plane (YB + 2 rows) staged per step, G in a 4-slot ring; the next
// step's slabs and the next k-step's operands are in flight while the MFMAs run.
struct Zf1Args {
  const float* G;
  const float* X;
  float* dW;
  float* part;  // non-null: per-workgroup partial tiles (k_wgrad_reduce) instead of atomics
  int N, M, Cc, D, H, W;
  int YB, nyb, ZS, zlen;
  int GR, GM, GS;  // G: row pitch, channel pitch, slot pitch (floats)
  int XR, XC, XS;  // X: row pitch (data at col 4), channel pitch, slot pitch
};

template <int YB, int WV>  // input rows per block, W <= 4 WV
__global__ __launch_bounds__(256) void k_conv3d_wgrad_zf1(Zf1Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H, D = a.D, M = a.M, Cc = a.Cc;
  float* gsl = smem;               // [4 slots][m][YB + 2 rows][GR]
  float* xsl = smem + 4 * a.GS;    // [2 slots][c][YB rows][XR], x at col x + 4
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int y0 = yb * YB;
  const int z0 = zs * a.zlen, z1 = min(D, z0 + a.zlen);
  for (int i = tid; i < 4 * a.GS + 2 * a.XS; i += 256) smem[i] = 0.f;  // halos and absent rows stay 0
  const int64_t plane = (int64_t)H * W, plane4 = plane / 4;
  const float* Gb = a.G + (int64_t)n * M * D * plane;
  const float* Xb = a.X + (int64_t)n * Cc * D * plane;
  const int W4v = W >> 2;
  constexpr int NXL = (5 * YB * WV + 255) / 256, NGL = (3 * (YB + 2) * WV + 255) / 256;
  int xg[NXL], xl[NXL], gg[NGL], gl[NGL];
#pragma unroll
  for (int j = 0; j < NXL; ++j) {
    const int i = tid + 256 * j;
    const int q = i % W4v, t = i / W4v, yy = t % YB, c = t / YB;
    const bool ok = c < Cc && y0 + yy < H;
    xg[j] = ok ? (int)(((int64_t)c * D) * plane4 + ((y0 + yy) * W + 4 * q) / 4) : -1;
    xl[j] = c * a.XC + yy * a.XR + 4 + 4 * q;
  }
#pragma unroll
  for (int j = 0; j < NGL; ++j) {
    const int i = tid + 256 * j;
    const int q = i % W4v, t = i / W4v, r = t % (YB + 2), m = t / (YB + 2);
    const int y = y0 - 1 + r;
    const bool ok = m < M && y >= 0 && y < H;
    gg[j] = ok ? (int)(((int64_t)m * D) * plane4 + (y * W + 4 * q) / 4) : -1;
    gl[j] = m * a.GM + r * a.GR + 4 * q;
  }
  // the slabs of the next ZP steps are in flight in registers (a step's MFMAs take less than an HBM
  // round trip): set p holds X[zi] and G[zi + 1] for the steps zi = p (mod ZP)
  constexpr int ZP = 3;
  float4 rx[ZP][NXL], rg[ZP][NGL];
  auto load_x = [&](int zi, float4 (&r)[NXL]) {  // (planes past the segment: clamped, never stored)
    const float4* src = reinterpret_cast<const float4*>(Xb) + (int64_t)(zi < D ? zi : D - 1) * plane4;
#pragma unroll
    for (int j = 0; j < NXL; ++j) {
      const float4 v = src[xg[j] < 0 ? 0 : xg[j]];
      r[j] = xg[j] < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : v;
    }
  };
  auto store_x = [&](int slot, const float4 (&r)[NXL]) {
#pragma unroll
    for (int j = 0; j < NXL; ++j)
      if (xg[j] >= 0) *reinterpret_cast<float4*>(xsl + slot * a.XS + xl[j]) = r[j];
  };
  // (zero-selects at the load here: with three steps' slabs in flight the early wait costs nothing, and
  // the store-side selects of k_conv3d_wgrad_zm measured slower for this kernel, 410 -> 430 us)
  auto load_g = [&](int pz, float4 (&r)[NGL]) {  // G plane pz (zero outside [0, D))
    const bool in = pz >= 0 && pz < D;
    const float4* src = reinterpret_cast<const float4*>(Gb) + (int64_t)(in ? pz : 0) * plane4;
#pragma unroll
    for (int j = 0; j < NGL; ++j) {
      const float4 v = src[gg[j] < 0 ? 0 : gg[j]];
      r[j] = (in && gg[j] >= 0) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_g = [&](int slot, const float4 (&r)[NGL], int) {
#pragma unroll
    for (int j = 0; j < NGL; ++j)
      if (gg[j] >= 0) *reinterpret_cast<float4*>(gsl + slot * a.GS + gl[j]) = r[j];
  };
  __syncthreads();
  load_g(z0 - 1, rg[0]);
  store_g((z0 + 3) & 3, rg[0], z0 - 1);
  load_g(z0, rg[0]);
  store_g(z0 & 3, rg[0], z0);
#pragma unroll
  for (int p = 0; p < ZP; ++p) {
    load_x(z0 + p, rx[p]);
    load_g(z0 + p + 1, rg[p]);
  }
  // lane roles: A rows r = 16 t + (lane & 15) -> (m, tz, ty); B column (c, tx) = lane & 15; k = lane >> 4
  const int li = lane & 15, lk = lane >> 4;
  int atz[2], aoff[2];
  bool aok[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int r = 16 * t + li, m = r / 9, tz = (r / 3) % 3, ty = r % 3;
    aok[t] = m < M;
    atz[t] = tz;
    aoff[t] = aok[t] ? m * a.GM + (2 - ty) * a.GR + lk : 0;  // G row y0 - 1 + (yy - ty + 2)
  }
  const int bc = li / 3, btx = li - 3 * bc;
  const bool bok = bc < Cc;
  const int boff = bok ? bc * a.XC + 3 + btx + lk : 0;  // X col px + tx - 1 at +4
  const int kpr = W >> 2, np = 4 / YB, yy = wave % YB, part = wave / YB;
  const int kb = (kpr * part) / np, ke = (kpr * (part + 1)) / np;
  f32x4 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) acc[0][t] = acc[1][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](int zi, float4 (&rxp)[NXL], float4 (&rgp)[NGL]) {
    store_x(zi & 1, rxp);
    store_g((zi + 1) & 3, rgp, zi + 1);
    __syncthreads();
    if (zi + ZP < z1) {
      load_x(zi + ZP, rxp);
      load_g(zi + ZP + 1, rgp);
    }
    // G plane qz - tz + 1 sits in slot (zi + 1 - tz) & 3
    const float* ga0 = gsl + ((zi + 1 - atz[0]) & 3) * a.GS + aoff[0] + yy * a.GR;
    const float* ga1 = gsl + ((zi + 1 - atz[1]) & 3) * a.GS + aoff[1] + yy * a.GR;
    const float* xb = xsl + (zi & 1) * a.XS + boff + yy * a.XR;
    auto ld = [&](int k, float& v0, float& v1, float& u) {
      const int px = 4 * (k < ke ? k : ke - 1);
      v0 = aok[0] ? ga0[px] : 0.f;
      v1 = aok[1] ? ga1[px] : 0.f;
      u = bok ? xb[px] : 0.f;
    };
    if (kb < ke) {
      float p0, p1, pu, q0, q1, qu;
      ld(kb, p0, p1, pu);
      int k = kb;
      for (; k + 1 < ke; k += 2) {
        ld(k + 1, q0, q1, qu);
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(p0, pu, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(p1, pu, acc[0][1], 0, 0, 0);
        ld(k + 2, p0, p1, pu);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(q0, qu, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(q1, qu, acc[1][1], 0, 0, 0);
      }
      if (k < ke) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(p0, pu, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(p1, pu, acc[0][1], 0, 0, 0);
      }
    }
  };
  for (int zi = z0; zi < z1; zi += ZP) {
    step(zi, rx[0], rg[0]);
    if (zi + 1 < z1) step(zi + 1, rx[1], rg[1]);
    if (zi + 2 < z1) step(zi + 2, rx[2], rg[2]);
  }
  __syncthreads();
  float* red = smem;  // [2 tiles][4 waves][4 rr][64 lanes]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[((t * 4 + wave) * 4 + rr) * 64 + lane] = acc[0][t][rr] + acc[1][t][rr];
  __syncthreads();
  float* pt = a.part ? a.part + (int64_t)blockIdx.x * (M * Cc * 27) : nullptr;
  for (int e = tid; e < 2 * 4 * 64; e += 256) {  // e = (t, rr, lane)
    const int ln = e & 63, rr = (e >> 6) & 3, t = e >> 8;
    const int r = 16 * t + 4 * (ln >> 4) + rr, col = ln & 15;
    const int m = r / 9, c = col / 3;
    if (m >= M || c >= Cc) continue;
    const int tz = (r / 3) % 3, ty = r % 3, tx = col - 3 * c;
    const float v = red[((t * 4 + 0) * 4 + rr) * 64 + ln] + red[((t * 4 + 1) * 4 + rr) * 64 + ln] +
                    red[((t * 4 + 2) * 4 + rr) * 64 + ln] + red[((t * 4 + 3) * 4 + rr) * 64 + ln];
    if (pt) pt[(m * Cc + c) * 27 + tz * 9 + ty * 3 + tx] = v;  // every (m < M, c < Cc) entry once
    else atomicAdd(&a.dW[((int64_t)m * Cc + c) * 27 + tz * 9 + ty * 3 + tx], v);
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
  // two blocks per CU over the whole chip, never more chunks than exist
  constexpr int target = 512;
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
  constexpr int yb_max = 4;  // 3->3 at 2x240x240x160: YB 8 / 512 blocks 530 us, YB 4 / 1024 blocks 462 us
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
  constexpr int target = 1024;
  int64_t gx = target;
  if (gx > a.nchunks) gx = a.nchunks;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(k_conv3d_wgrad_mz<SEG>, dim3((unsigned)gx), dim3(NT), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

bool use_mz(int M, int Cc, int stride) {
  constexpr bool on = true;
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
  constexpr int yb_max = 8;
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


// z-marching stride-1 kernel (k_conv3d_wgrad_zm): 16-channel tiles, W % 4 == 0 (16-B rows), W <= 80,
// at least 8 output and 8 input channels (the few-channel layers keep their own tilings)
bool use_zm(int M, int Cc, int stride, int Do, int Ho, int Wo, int Di, int Hi, int Wi, const void* G, const void* X) {
  constexpr bool on = true;
  return on && stride == 1 && M >= 8 && Cc >= 8 && Do == Di && Ho == Hi && Wo == Wi && Wo % 4 == 0 && Wo <= 80 &&
         (reinterpret_cast<uintptr_t>(G) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

int zm_setup(ZmArgs& a, size_t& lds, dim3& grid, int N, int M, int Cc, int D, int H, int W, int ncu) {
  a.N = N; a.M = M; a.Cc = Cc; a.D = D; a.H = H; a.W = W;
  a.W4 = W;  // W % 4 == 0
  a.PX = ((W + 3 + 1) / 2) * 2;  // cols 0..W + 2 (data at 2..W + 1), even (8-B stores)
  a.YB = 0;
  for (int yb : {4, 2}) {  // rows per block: the first tiling that fits
    const int ms = pad_mod32(yb * a.W4, 2), rx = pad_mod32((yb + 2) * a.PX, 2);
    const size_t bytes = (size_t)4 * (4 * 16 * ms + 2 * 16 * rx);
    if (bytes <= 163840) {
      a.YB = yb; a.MS = ms; a.RX = rx;
      lds = bytes > ZM_RED_BYTES ? bytes : ZM_RED_BYTES;  // the end's 2-wave reduction image: 55.3 KB
      if (lds < 81920 + 16) lds = 81920 + 16;  // one block per CU (two 4-wave blocks measured slower: 212 -> 281 us at 32 -> 32)
      break;
    }
  }
  if (!a.YB) return TB_ERR_UNSUPPORTED_SIZE;
  a.nyb = (H + a.YB - 1) / a.YB;
  a.mtiles = (M + 15) / 16;
  a.ctiles = (Cc + 15) / 16;
  // z segments: the launch takes ceil(blocks / (CUs x blocks per CU)) rounds of zlen + 2 plane steps
  // (two ring-fill planes per segment): the segment length minimising that
  const int per_cu = 1;
  const int base = N * a.nyb * a.mtiles * a.ctiles;
  int best = 1 << 30;
  a.zlen = D;
  for (int zl = D; zl >= 4 || zl == D; --zl) {
    const int zs = (D + zl - 1) / zl;
    const int rounds = (base * zs + ncu * per_cu - 1) / (ncu * per_cu);
    const int cost = rounds * (zl + 2);
    if (cost < best) {
      best = cost;
      a.zlen = zl;
    }
    if (zl <= 1) break;
  }
  a.ZS = (D + a.zlen - 1) / a.zlen;
  grid = dim3((unsigned)(N * a.nyb * a.ZS), (unsigned)(a.mtiles * a.ctiles));
  return TB_OK;
}

// 8 waves per block (one block per CU: two waves per SIMD; 4-wave blocks two per CU measured slower,
// 4-wave blocks one per CU 7 -- 20 us slower per call)
int launch_zm(const ZmArgs& a, size_t lds, dim3 grid, hipStream_t st) {
  auto kern = a.W > 40 ? (a.YB == 4 ? k_conv3d_wgrad_zm<4, 20, 8> : k_conv3d_wgrad_zm<2, 20, 8>)
                       : (a.YB == 4 ? k_conv3d_wgrad_zm<4, 10, 8> : k_conv3d_wgrad_zm<2, 10, 8>);
  const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, grid, dim3(512), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

// stride-2 z-marching kernel (k_conv3d_wgrad_zm2): >= 8 input channels, Wo % 4 == 0, Wo <= 40,
// input rows of exactly 2 Wo (padding 1)
bool use_zm2(int M, int Cc, int stride, int Do, int Ho, int Wo, int Di, int Hi, int Wi, const void* G, const void* X) {
  constexpr bool on = true;
  return on && stride == 2 && M >= 8 && Cc >= 8 && Wo % 4 == 0 && Wo <= 40 && Wi == 2 * Wo && Hi == 2 * Ho &&
         Di == 2 * Do && (reinterpret_cast<uintptr_t>(G) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

int zm2_setup(Zm2Args& a, size_t& lds, dim3& grid, int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi,
              int Wi, int ncu) {
  a.N = N; a.M = M; a.Cc = Cc; a.Do = Do; a.Ho = Ho; a.Wo = Wo; a.Di = Di; a.Hi = Hi; a.Wi = Wi;
  a.PX = ((2 * Wo + 3 + 1) / 2) * 2;
  constexpr int yb_env = 0;  // rows per block: the first tiling that fits (below)
  a.YB = 0;
  for (int yb : {2, 1}) {  // two output rows per block where the ring fits: twice the MFMAs per staged plane
    if ((yb_env && yb != yb_env) || yb > Ho) continue;
    for (int rem : {2, 4}) {  // X channel pitch mod 32: 2 (2-way B conflicts), 4 (tighter pad)
      const int rx = pad_mod32((2 * yb + 1) * a.PX, rem), ms = pad_mod32(yb * Wo, 2);
      const size_t ring = (size_t)4 * (2 * 32 * ms + 5 * 16 * rx), red = (size_t)4 * 2 * 27 * 4 * 64;
      const size_t need = ring > red ? ring : red;
      if (need <= 163840) {
        a.YB = yb; a.RX = rx; a.MS = ms;
        lds = need;
        break;
      }
    }
    if (a.YB) break;
  }
  if (!a.YB) return TB_ERR_UNSUPPORTED_SIZE;
  a.nyb = (Ho + a.YB - 1) / a.YB;
  a.mtiles = (M + 31) / 32;
  a.ctiles = (Cc + 15) / 16;
  const int base = N * a.nyb * a.mtiles * a.ctiles;
  const int per_cu = 1;  // 8-wave blocks: two waves per SIMD already
  int best = 1 << 30;
  a.zlen = Do;
  for (int zl = Do; zl >= 1; --zl) {
    const int zs = (Do + zl - 1) / zl;
    const int rounds = (base * zs + per_cu * ncu - 1) / (per_cu * ncu);
    const int cost = rounds * (zl + 1);
    if (cost < best) {
      best = cost;
      a.zlen = zl;
    }
  }
  a.ZS = (Do + a.zlen - 1) / a.zlen;
  grid = dim3((unsigned)(N * a.nyb * a.ZS), (unsigned)(a.mtiles * a.ctiles));
  return TB_OK;
}

int launch_zm2(const Zm2Args& a, size_t lds, dim3 grid, hipStream_t st) {
  auto kern = a.YB == 2 ? (a.Wo <= 20 ? k_conv3d_wgrad_zm2<2, 5, 8> : k_conv3d_wgrad_zm2<2, 10, 8>)
                        : (a.Wo <= 20 ? k_conv3d_wgrad_zm2<1, 5, 8> : k_conv3d_wgrad_zm2<1, 10, 8>);
  const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, grid, dim3(512), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

// few-channel stride-2 kernel (k_conv3d_wgrad_zf2): Cc <= 5, Wo % 4 == 0, Wo <= 80, 2x input rows
bool use_zf2(int M, int Cc, int stride, int Do, int Ho, int Wo, int Di, int Hi, int Wi, const void* G, const void* X) {
  constexpr bool on = true;
  return on && stride == 2 && Cc <= 5 && Wo % 4 == 0 && Wo <= 80 && Wi == 2 * Wo && Hi == 2 * Ho && Di == 2 * Do &&
         (reinterpret_cast<uintptr_t>(G) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

int zf2_setup(Zf2Args& a, int& MT, size_t& lds, dim3& grid, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
              int Hi, int Wi, int ncu) {
  a.N = N; a.M = M; a.Cc = Cc; a.Do = Do; a.Ho = Ho; a.Wo = Wo; a.Di = Di; a.Hi = Hi; a.Wi = Wi;
  MT = M > 16 ? 2 : 1;
  a.PX = ((2 * Wo + 3 + 1) / 2) * 2;
  a.YB = 0;
  for (int yb : {4, 2, 1}) {
    const int rx = pad_mod32((2 * yb + 1) * a.PX, 8), ms = pad_mod32(yb * Wo, 2);
    const size_t ring = (size_t)4 * (2 * 16 * MT * ms + 5 * Cc * rx), red = (size_t)4 * MT * 9 * 8 * 4 * 64;
    const size_t need = ring > red ? ring : red;
    if (need <= 163840) {
      a.YB = yb; a.RX = rx; a.MS = ms;
      lds = need;
      break;
    }
  }
  if (!a.YB) return TB_ERR_UNSUPPORTED_SIZE;
  a.nyb = (Ho + a.YB - 1) / a.YB;
  a.mtiles = (M + 16 * MT - 1) / (16 * MT);
  const int base = N * a.nyb * a.mtiles;
  int best = 1 << 30;
  a.zlen = Do;
  for (int zl = Do; zl >= 1; --zl) {
    const int zs = (Do + zl - 1) / zl;
    const int rounds = (base * zs + ncu - 1) / ncu;
    const int cost = rounds * (zl + 1);
    if (cost < best) {
      best = cost;
      a.zlen = zl;
    }
  }
  a.ZS = (Do + a.zlen - 1) / a.zlen;
  grid = dim3((unsigned)(N * a.nyb * a.ZS), (unsigned)a.mtiles);
  return TB_OK;
}

template <int YB, int MT>
int launch_zf2_t(const Zf2Args& a, size_t lds, dim3 grid, hipStream_t st) {
  auto kern = a.Wo <= 40 ? k_conv3d_wgrad_zf2<YB, MT, 10, 8> : k_conv3d_wgrad_zf2<YB, MT, 20, 8>;
  const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, grid, dim3(512), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}
int launch_zf2(const Zf2Args& a, int MT, size_t lds, dim3 grid, hipStream_t st) {
  if (MT == 1) return a.YB == 4 ? launch_zf2_t<4, 1>(a, lds, grid, st) : a.YB == 2 ? launch_zf2_t<2, 1>(a, lds, grid, st) : launch_zf2_t<1, 1>(a, lds, grid, st);
  return a.YB == 4 ? launch_zf2_t<4, 2>(a, lds, grid, st) : a.YB == 2 ? launch_zf2_t<2, 2>(a, lds, grid, st) : launch_zf2_t<1, 2>(a, lds, grid, st);
}

// few-channel stride-1 z-marching kernel (k_conv3d_wgrad_zf1): 9 M <= 32, 3 Cc <= 16, W % 4 == 0
bool use_zf1(int M, int Cc, int stride, int Do, int Ho, int Wo, int Di, int Hi, int Wi, const void* G, const void* X) {
  constexpr bool on = true;
  return on && stride == 1 && M <= 3 && Cc <= 5 && Do == Di && Ho == Hi && Wo == Wi && Wo % 4 == 0 && Wo <= 256 &&
         (reinterpret_cast<uintptr_t>(G) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

int zf1_setup(Zf1Args& a, size_t& lds, dim3& grid, int N, int M, int Cc, int D, int H, int W, int ncu) {
  a.N = N; a.M = M; a.Cc = Cc; a.D = D; a.H = H; a.W = W;
  constexpr int yb_env = 0;  // rows per block: the first tiling that fits (below)
  // pitches: rows of one G channel 4 banks apart, channels and slots spread over the banks
  a.GR = pad_mod32(W, 4);
  a.XR = pad_mod32(W + 8, 4);
  a.YB = 0;
  for (int yb : {2, 4, 1}) {
    if (yb_env && yb != yb_env) continue;
    const int gm = pad_mod32((yb + 2) * a.GR, 12), gs = pad_mod32(M * gm, 20);
    const int xc = pad_mod32(yb * a.XR, 8), xs = pad_mod32(Cc * xc, 16);
    const size_t bytes = (size_t)4 * (4 * gs + 2 * xs);
    if (bytes <= 81920) {  // two blocks per CU
      a.YB = yb; a.GM = gm; a.GS = gs; a.XC = xc; a.XS = xs;
      lds = bytes > (size_t)2 * 4 * 4 * 64 * 4 ? bytes : (size_t)2 * 4 * 4 * 64 * 4;
      break;
    }
  }
  if (!a.YB) return TB_ERR_UNSUPPORTED_SIZE;
  a.nyb = (H + a.YB - 1) / a.YB;
  // z segments: two blocks per CU; ceil(blocks / (2 CUs)) rounds of zlen + 2 plane steps
  const int base = N * a.nyb;
  int best = 1 << 30;
  a.zlen = D;
  for (int zl = D; zl >= 1; --zl) {
    const int zs = (D + zl - 1) / zl;
    const int rounds = (base * zs + 2 * ncu - 1) / (2 * ncu);
    const int cost = rounds * (zl + 2);
    if (cost < best) {
      best = cost;
      a.zlen = zl;
    }
  }
  a.ZS = (D + a.zlen - 1) / a.zlen;
  grid = dim3((unsigned)(N * a.nyb * a.ZS));
  return TB_OK;
}

template <int YB>
int launch_zf1_t(const Zf1Args& a, size_t lds, dim3 grid, hipStream_t st) {
  auto kern = a.W <= 128 ? k_conv3d_wgrad_zf1<YB, 32>
                         : a.W <= 160 ? k_conv3d_wgrad_zf1<YB, 40> : k_conv3d_wgrad_zf1<YB, 64>;
  const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

int launch_zf1(const Zf1Args& a, size_t lds, dim3 grid, hipStream_t st) {
  return a.YB == 4 ? launch_zf1_t<4>(a, lds, grid, st) : a.YB == 2 ? launch_zf1_t<2>(a, lds, grid, st)
                                                                    : launch_zf1_t<1>(a, lds, grid, st);
}
}  // namespace

// dW (M x Cc x 27, zeroed here) of a 3x3x3 convolution with stride 1 or 2, padding 1 (file header).
int tb_conv3d_wgrad_f32(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
                        int Hi, int Wi, int stride, int pad, void* stream) {
  if (!G || !X || !dW) return TB_ERR_INVALID_ARG;
  hipStream_t st0 = reinterpret_cast<hipStream_t>(stream);
  if (pad == 1 && N >= 1 && use_zm(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X)) {
    static const int ncu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
      return n;
    }();
    ZmArgs z{};
    size_t lds = 0;
    dim3 grid;
    if (zm_setup(z, lds, grid, N, M, Cc, Do, Ho, Wo, ncu) == TB_OK) {
      z.G = G; z.X = X; z.dW = dW;
      if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * Cc * 27, st0) != hipSuccess) return TB_ERR_HIP;
      return launch_zm(z, lds, grid, st0);
    }
  }
  if (pad == 1 && N >= 1 && use_zm2(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X)) {
    static const int ncu2 = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
      return n;
    }();
    Zm2Args z{};
    size_t lds = 0;
    dim3 grid;
    if (zm2_setup(z, lds, grid, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, ncu2) == TB_OK) {
      z.G = G; z.X = X; z.dW = dW;
      if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * Cc * 27, st0) != hipSuccess) return TB_ERR_HIP;
      return launch_zm2(z, lds, grid, st0);
    }
  }
  if (pad == 1 && N >= 1 && use_zf1(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X)) {
    static const int ncu4 = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
      return n;
    }();
    Zf1Args z{};
    size_t lds = 0;
    dim3 grid;
    if (zf1_setup(z, lds, grid, N, M, Cc, Do, Ho, Wo, ncu4) == TB_OK) {
      z.G = G; z.X = X; z.dW = dW;
      if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * Cc * 27, st0) != hipSuccess) return TB_ERR_HIP;
      return launch_zf1(z, lds, grid, st0);
    }
  }
  if (pad == 1 && N >= 1 && use_zf2(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X)) {
    static const int ncu3 = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
      return n;
    }();
    Zf2Args z{};
    int MT = 1;
    size_t lds = 0;
    dim3 grid;
    if (zf2_setup(z, MT, lds, grid, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, ncu3) == TB_OK) {
      z.G = G; z.X = X; z.dW = dW;
      if (hipMemsetAsync(dW, 0, sizeof(float) * (size_t)M * Cc * 27, st0) != hipSuccess) return TB_ERR_HIP;
      return launch_zf2(z, MT, lds, grid, st0);
    }
  }
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

static int wgrad_ncu() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
    return c;
  }();
  return n;
}

// The z-marching route tb_conv3d_wgrad_f32 takes for these sizes, set up for partial tiles: the partial
// tile of each workgroup is TM x TC x 27 floats (k_wgrad_reduce), `blocks` workgroups per tile.
struct ZRoute {
  int kind = 0;  // 0: none (the general kernel, atomics), 1 zm, 2 zm2, 3 zf1, 4 zf2
  ZmArgs zm{};
  Zm2Args zm2{};
  Zf1Args zf1{};
  Zf2Args zf2{};
  int MT = 1;
  size_t lds = 0;
  dim3 grid;
  int TM = 0, TC = 0, ctiles = 1;
  size_t bytes() const { return kind ? (size_t)grid.x * grid.y * TM * TC * 27 * 4 : 0; }
};

static ZRoute zroute(int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi, int Wi, int stride, int pad,
                     const void* G, const void* X) {
  ZRoute r;
  if (pad != 1 || N < 1) return r;
  const int ncu = wgrad_ncu();
  if (use_zm(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X) &&
      zm_setup(r.zm, r.lds, r.grid, N, M, Cc, Do, Ho, Wo, ncu) == TB_OK) {
    r.kind = 1, r.TM = 16, r.TC = 16, r.ctiles = r.zm.ctiles;
  } else if (use_zm2(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X) &&
             zm2_setup(r.zm2, r.lds, r.grid, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, ncu) == TB_OK) {
    r.kind = 2, r.TM = 32, r.TC = 16, r.ctiles = r.zm2.ctiles;
  } else if (use_zf1(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X) &&
             zf1_setup(r.zf1, r.lds, r.grid, N, M, Cc, Do, Ho, Wo, ncu) == TB_OK) {
    r.kind = 3, r.TM = M, r.TC = Cc, r.ctiles = 1;
  } else if (use_zf2(M, Cc, stride, Do, Ho, Wo, Di, Hi, Wi, G, X) &&
             zf2_setup(r.zf2, r.MT, r.lds, r.grid, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, ncu) == TB_OK) {
    r.kind = 4, r.TM = 16 * r.MT, r.TC = Cc, r.ctiles = 1;
  }
  return r;
}

int64_t tb_conv3d_wgrad_ws_bytes(int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi, int Wi, int stride,
                                 int pad) {
  return (int64_t)zroute(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad, nullptr, nullptr).bytes();
}

int tb_conv3d_wgrad_ws_f32(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo,
                           int Di, int Hi, int Wi, int stride, int pad, void* ws, size_t ws_bytes, void* stream) {
  if (!G || !X || !dW) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ZRoute r = zroute(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad, G, X);
  if (!ws || !r.kind || ws_bytes < r.bytes() || (reinterpret_cast<uintptr_t>(ws) & 3) != 0)
    return tb_conv3d_wgrad_f32(G, X, dW, N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad, stream);
  float* part = static_cast<float*>(ws);
  int rc = TB_OK;
  switch (r.kind) {
    case 1: r.zm.G = G, r.zm.X = X, r.zm.dW = dW, r.zm.part = part; rc = launch_zm(r.zm, r.lds, r.grid, st); break;
    case 2: r.zm2.G = G, r.zm2.X = X, r.zm2.dW = dW, r.zm2.part = part; rc = launch_zm2(r.zm2, r.lds, r.grid, st); break;
    case 3: r.zf1.G = G, r.zf1.X = X, r.zf1.dW = dW, r.zf1.part = part; rc = launch_zf1(r.zf1, r.lds, r.grid, st); break;
    default: r.zf2.G = G, r.zf2.X = X, r.zf2.dW = dW, r.zf2.part = part; rc = launch_zf2(r.zf2, r.MT, r.lds, r.grid, st); break;
  }
  if (rc != TB_OK) return rc;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((r.TM * r.TC * 27 + 63) / 64, r.grid.y), dim3(1024), 0, st,
                     static_cast<const float*>(part), dW, (int)r.grid.x, r.TM, r.TC, r.ctiles, M, Cc);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
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
