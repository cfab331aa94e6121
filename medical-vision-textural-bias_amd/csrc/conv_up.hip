// conv_up.hip -- the U-Net's full-resolution stride-2 layers with few channels on one side.
//
// The reference's MONAI UNet (10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199) enters with
// Conv3d(4 -> 16, stride 2) twice (the first unit and its residual) and leaves with
// ConvTranspose3d(32 -> 3, stride 2, output_padding 1).  MIOpen runs these through layout transposes
// and im2col / col2im GEMMs (467 us per forward of the entry conv, 1.17 ms for the transposed
// forward, 0.82 ms for its input gradient per C3 step).  All three are one of two stencils:
//
//   k_conv_s2_fewin    out[m][o] = b[m] + sum_{c, t} K[c][t][m] in[c][2 o + t - 1]      (c < CIN <= 4)
//     * Conv3d(4 -> 16, s2) forward: in = x, K[c][t][m] = W[m][c][t];
//     * the input gradient of ConvTranspose3d(32 -> 3, s2): in = dY (3 channels), out = dX (32),
//       K[c][t][m] = W[m][c][t] with W the transposed conv's [Cin = m][Cout = c] weight;
//   k_convT_fewout     y[m][2 j + p] = b[m] + sum_c sum_{(d, t) in S(p)} W[c][m][t] x[c][j + d]   (m < MO <= 4)
//     per axis S(0) = {(0, 1)}, S(1) = {(0, 2), (1, 0)}: the 8 output parities of one input position
//     from its 2 x 2 x 2 neighbourhood (sub-pixel form: every multiply-add is a real tap).
//
// Both march along z with the input planes staged in an LDS ring and the next step's planes in
// registers; one thread per output position (A) or input position (B) holds all output channels
// (A: its 27 CIN inputs in registers, packed FMAs per output pair; B: the 8 parities x MO channels);
// the weights are scalar loads (SGPR operands).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "texbias.h"

namespace {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// Weights are wave-uniform: read through the constant address space they become scalar loads and
// SGPR operands of the FMAs (as broadcast LDS reads they cost an LDS instruction per 2 FMAs: the
// first version of these kernels was LDS-bound at 8 % of the FMA rate).
typedef const __attribute__((address_space(4))) float* cfloat_p;
typedef const __attribute__((address_space(4))) f2v* cf2v_p;

// ------------------------------------------------------------------------------ stride-2 conv
struct S2Args {
  const float* in;
  const float* K;     // [MOUT / 2][CIN 27][2]: output channel pairs
  const float* bias;  // [MOUT] or null
  float* out;
  int Do, Ho, Wo, Di, Hi, Wi;
  int ZS, zlen, nyb;
  int PX, RR;  // LDS row pitch; rows per channel slab (2 TY + 1)
};

// NTH = 512: the two halves of the block share the positions and split the output pairs (registers of
// the 27 CIN inputs + half the accumulators: two waves per SIMD instead of one for CIN = 4, MOUT = 32)
template <int CIN, int MOUT, int TY, int WV, int NTH = 256>  // WV: most float4 per input row (Wi <= 4 WV)
__global__ __launch_bounds__(NTH) void k_conv_s2_fewin(S2Args a) {
  static_assert(MOUT % 2 == 0, "packed output pairs");
  constexpr int NHALF = NTH / 256, MP = MOUT / 2 / NHALF;  // output pairs per half
  constexpr int NR = 2 * TY + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x;
  constexpr int PX = 4 * WV + 12, SS = CIN * NR * PX;  // row pitch (odd multiple of 4), slot stride
  // [3][CIN][NR][PX], input column xi at xi + 4: step z reads planes 2z - 1 .. 2z + 1; its first stores
  // put planes 2z, 2z + 1 over the slots of 2z - 3, 2z - 2 (three slots instead of five: 58 KB at the
  // C3 shapes, two blocks per CU)
  float* ring = smem;
  for (int i = tid; i < 3 * SS; i += NTH) ring[i] = 0.f;  // halos, padding rows stay 0
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int y0 = yb * TY;
  const int z0 = zs * a.zlen, z1 = min(a.Do, z0 + a.zlen);
  const int Di = a.Di, Hi = a.Hi, Wi = a.Wi;
  const int64_t iplane = (int64_t)Hi * Wi, iplane4 = iplane / 4;
  const float4* inb = reinterpret_cast<const float4*>(a.in + (int64_t)n * CIN * Di * iplane);
  // staging items of one plane: (c, r, q) -> input row 2 y0 - 1 + r, float4 q
  const int W4 = Wi >> 2;
  constexpr int NL = (CIN * NR * WV + NTH - 1) / NTH;
  int gof[NL], lof[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + NTH * j;
    const int q = i % W4, t = i / W4, r = t % NR, c = t / NR;
    const int yi = 2 * y0 - 1 + r;
    const bool ok = c < CIN && yi >= 0 && yi < Hi;
    gof[j] = ok ? (int)((int64_t)c * Di * iplane4 + ((int64_t)yi * Wi + 4 * q) / 4) : -1;
    lof[j] = (c * NR + r) * PX + 4 + 4 * q;
  }
  float4 ra[NL], rb[NL];
  auto load = [&](int zi, float4 (&r)[NL]) {
    const bool in = zi >= 0 && zi < Di;
    const float4* src = inb + (int64_t)(in ? zi : 0) * iplane4;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      r[j] = src[gof[j] < 0 ? 0 : gof[j]];  // zeroed at the store (a select here waits for the load)
    }
  };
  auto store = [&](int zi, const float4 (&r)[NL]) {
    float* d = ring + ((zi + 3) % 3) * SS;
    const bool in = zi >= 0 && zi < Di;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      if (gof[j] >= 0) *reinterpret_cast<float4*>(d + lof[j]) = in ? r[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  __syncthreads();  // zero fill before any slab store
  load(2 * z0 - 1, ra);
  store(2 * z0 - 1, ra);
  load(2 * z0, ra);
  load(2 * z0 + 1, rb);
  // this thread's output position: row y0 + oy, column ox; output pairs mh * MP .. + MP - 1
  const int pt = tid & 255, mh = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int Wo = a.Wo, oy = pt / Wo, ox = pt - oy * Wo;
  const bool act = oy < TY && y0 + oy < a.Ho;
  const int roff = (2 * oy) * PX + 2 * ox + 3;  // + (ty PX + tx): input row 2 oy + ty, column 2 ox + tx - 1
  f2v bias2[MP];
#pragma unroll
  for (int mm = 0; mm < MP; ++mm) {
    const int m = mh * MP + mm;
    bias2[mm] = a.bias ? f2v{a.bias[2 * m], a.bias[2 * m + 1]} : f2v{0.f, 0.f};
  }
  const int64_t oplane = (int64_t)a.Ho * Wo;
  float* outb = a.out + (int64_t)n * MOUT * a.Do * oplane + (int64_t)(y0 + oy) * Wo + ox;
  // LATE (the 256-thread form): outputs leave one step late (pend), after the next planes' loads, so the
  // wait for those loads at the next step's LDS store never includes a store issued in the same step
  // (3 -> 32: 225 -> 212 us; the 512-thread 4 -> 32 form measured 278 -> 317 us with it: immediate stores)
  constexpr bool LATE = NTH == 256;
  f2v pend[MP];
  auto put = [&](int zp) {
    float* o = outb + (int64_t)zp * oplane;
#pragma unroll
    for (int mm = 0; mm < MP; ++mm) {
      const int m = mh * MP + mm;
      o[(int64_t)(2 * m) * a.Do * oplane] = pend[mm].x;
      o[(int64_t)(2 * m + 1) * a.Do * oplane] = pend[mm].y;
    }
  };
  for (int z = z0; z < z1; ++z) {
    store(2 * z, ra);
    store(2 * z + 1, rb);
    __syncthreads();
    if (LATE || z + 1 < z1) {  // (LATE: unconditionally; past the segment: never stored)
      load(2 * z + 2, ra);
      load(2 * z + 3, rb);
    }
    if (LATE && act && z > z0) put(z - 1);
    if (act) {
      // the position's 27 CIN inputs into registers, then one packed FMA chain per output pair
      float v[CIN * 27];
#pragma unroll
      for (int tz = 0; tz < 3; ++tz) {
        const float* sl = ring + ((2 * z - 1 + tz + 3) % 3) * SS + roff;
#pragma unroll
        for (int c = 0; c < CIN; ++c)
#pragma unroll
          for (int ty = 0; ty < 3; ++ty)
#pragma unroll
            for (int tx = 0; tx < 3; ++tx) v[c * 27 + tz * 9 + ty * 3 + tx] = sl[(c * NR + ty) * PX + tx];
      }
      const cf2v_p kp = (cf2v_p)(cfloat_p)a.K;
#pragma unroll
      for (int mm = 0; mm < MP; ++mm) {
        const int m = mh * MP + mm;
        f2v acc = bias2[mm];
#pragma unroll
        for (int k = 0; k < CIN * 27; ++k) acc = __builtin_elementwise_fma(f2v{v[k], v[k]}, kp[m * CIN * 27 + k], acc);
        if (LATE) {
          pend[mm] = acc;
        } else {
          float* o = outb + (int64_t)z * oplane;
          o[(int64_t)(2 * m) * a.Do * oplane] = acc.x;
          o[(int64_t)(2 * m + 1) * a.Do * oplane] = acc.y;
        }
      }
    }
    __syncthreads();  // every wave is done with this step's slots before the next step's stores
  }
  if (LATE && act && z1 > z0) put(z1 - 1);
}

// --------------------------------------------------------------- ConvTranspose3d, few outputs
struct TArgs {
  const float* x;
  const float* W;     // [Cin][MO][27] (the module's own weight layout)
  const float* bias;  // [MO] or null
  float* y;
  int Cin, Di, Hi, Wi;
  int ZS, zlen, nyb;
  int PX, CS;  // LDS row pitch, channel slab stride (TY + 1 rows)
};

template <int MO, int TY, int WV, int NTH = 256, int U = 1>  // U: input channels per FMA-loop iteration
__global__ __launch_bounds__(NTH) void k_convT_fewout(TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x;
  constexpr int PX = 4 * WV + 8, CS = (TY + 1) * PX;
  const int Cin = a.Cin, SS = Cin * CS;
  // [2][Cin][TY + 1][PX], column xi at xi + 4 (xi = Wi: zero): step z reads planes z, z + 1; its first
  // store puts plane z + 1 over the slot of z - 1
  float* ring = smem;
  for (int i = tid; i < 2 * SS; i += NTH) ring[i] = 0.f;
  const cfloat_p wg = (cfloat_p)a.W;  // [Cin][MO][27], scalar loads
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int y0 = yb * TY;
  const int Di = a.Di, Hi = a.Hi, Wi = a.Wi;
  const int z0 = zs * a.zlen, z1 = min(Di, z0 + a.zlen);
  const int64_t iplane = (int64_t)Hi * Wi, iplane4 = iplane / 4;
  const float4* xb = reinterpret_cast<const float4*>(a.x + (int64_t)n * Cin * Di * iplane);
  const int W4 = Wi >> 2;
  // staging items of one plane: (c, r, q) -> input row y0 + r (r <= TY), float4 q; at most 32 channels
  constexpr int NL = (32 * (TY + 1) * WV + NTH - 1) / NTH;
  const int nitem = Cin * (TY + 1) * W4;
  int gof[NL], lof[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + NTH * j;
    const int q = i % W4, t = i / W4, r = t % (TY + 1), c = t / (TY + 1);
    const int yi = y0 + r;
    const bool ok = i < nitem && yi < Hi;
    gof[j] = ok ? (int)((int64_t)c * Di * iplane4 + ((int64_t)yi * Wi + 4 * q) / 4) : -1;
    lof[j] = c * CS + r * PX + 4 + 4 * q;
  }
  float4 rg[NL];
  auto load = [&](int zi) {
    const bool in = zi < Di;
    const float4* src = xb + (int64_t)(in ? zi : 0) * iplane4;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      rg[j] = src[gof[j] < 0 ? 0 : gof[j]];  // zeroed at the store (a select here waits for the load)
    }
  };
  auto store = [&](int zi) {
    float* d = ring + (zi & 1) * SS;
    const bool in = zi < Di;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      if (gof[j] >= 0) *reinterpret_cast<float4*>(d + lof[j]) = in ? rg[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  __syncthreads();
  load(z0);
  store(z0);
  load(z0 + 1);
  const int jy = tid / Wi, jx = tid - jy * Wi;
  const bool act = jy < TY && y0 + jy < Hi;
  const int roff = jy * PX + jx + 4;
  const int Ho = 2 * Hi, Wo = 2 * Wi, Do = 2 * Di;
  const int64_t oplane = (int64_t)Ho * Wo;
  float bia[MO];
#pragma unroll
  for (int m = 0; m < MO; ++m) bia[m] = a.bias ? a.bias[m] : 0.f;
  float* yb0 = a.y + (int64_t)n * MO * Do * oplane + (int64_t)(2 * (y0 + jy)) * Wo + 2 * jx;
  // (outputs one step late, as k_conv_s2_fewin's 256-thread form: 291 -> 317 us here, not taken)
  for (int z = z0; z < z1; ++z) {
    store(z + 1);  // plane z + 1 (zero past Di)
    __syncthreads();
    if (z + 1 < z1) load(z + 2);
    // acc[m][pz][py][px]
    float acc[MO][2][2][2];
#pragma unroll
    for (int m = 0; m < MO; ++m)
#pragma unroll
      for (int p = 0; p < 8; ++p) acc[m][p >> 2][(p >> 1) & 1][p & 1] = bia[m];
    if (act) {
      const float* s0 = ring + (z & 1) * SS + roff;
      const float* s1 = ring + ((z + 1) & 1) * SS + roff;
#pragma unroll U
      for (int c = 0; c < Cin; ++c) {
        float v[2][2][2];  // [dz][dy][dx]
        v[0][0][0] = s0[c * CS];
        v[0][0][1] = s0[c * CS + 1];
        v[0][1][0] = s0[c * CS + PX];
        v[0][1][1] = s0[c * CS + PX + 1];
        v[1][0][0] = s1[c * CS];
        v[1][0][1] = s1[c * CS + 1];
        v[1][1][0] = s1[c * CS + PX];
        v[1][1][1] = s1[c * CS + PX + 1];
        const cfloat_p wc = wg + c * MO * 27;
#pragma unroll
        for (int m = 0; m < MO; ++m) {
          const cfloat_p wk = wc + m * 27;
          // per axis: parity 0 <- (d 0, t 1); parity 1 <- (d 0, t 2) + (d 1, t 0)
#pragma unroll
          for (int pz = 0; pz < 2; ++pz)
#pragma unroll
            for (int py = 0; py < 2; ++py)
#pragma unroll
              for (int px = 0; px < 2; ++px) {
                float s = acc[m][pz][py][px];
#pragma unroll
                for (int dz = 0; dz <= pz; ++dz)
#pragma unroll
                  for (int dy = 0; dy <= py; ++dy)
#pragma unroll
                    for (int dx = 0; dx <= px; ++dx) {
                      const int tz = pz ? (dz ? 0 : 2) : 1, ty = py ? (dy ? 0 : 2) : 1, tx = px ? (dx ? 0 : 2) : 1;
                      s = fmaf(v[dz][dy][dx], wk[tz * 9 + ty * 3 + tx], s);
                    }
                acc[m][pz][py][px] = s;
              }
        }
      }
#pragma unroll
      for (int m = 0; m < MO; ++m)
#pragma unroll
        for (int pz = 0; pz < 2; ++pz)
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            float* o = yb0 + ((int64_t)m * Do + 2 * z + pz) * oplane + (int64_t)py * Wo;
            *reinterpret_cast<float2*>(o) = make_float2(acc[m][pz][py][0], acc[m][pz][py][1]);
          }
    }
    __syncthreads();
  }
}

int ncu_count() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
    return c;
  }();
  return n;
}

// z segment length for `base` blocks per z segment, `per_cu` blocks resident per CU: rounds x (len + fill)
int zseg(int D, int base, int per_cu, int fill) {
  const int slots = per_cu * ncu_count();
  int best = 1 << 30, zl = D;
  for (int l = D; l >= 1; --l) {
    const int zs = (D + l - 1) / l, rounds = (base * zs + slots - 1) / slots, cost = rounds * (l + fill);
    if (cost < best) best = cost, zl = l;
  }
  return zl;
}

template <int CIN, int MOUT, int WV>
int launch_s2(S2Args& a, size_t lds, int N, hipStream_t st) {
  constexpr int TY = 3;
  // CIN = 4, MOUT = 32 (the stacked entry unit + residual): 512 threads splitting the output pairs
  constexpr int NT = (CIN == 4 && MOUT == 32) ? 512 : 256;
  auto kern = k_conv_s2_fewin<CIN, MOUT, TY, WV, NT>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  const int per_cu = lds <= 81920 ? 2 : 1;
  a.zlen = zseg(a.Do, N * a.nyb, per_cu, 1);
  a.ZS = (a.Do + a.zlen - 1) / a.zlen;
  hipLaunchKernelGGL(kern, dim3((unsigned)(N * a.nyb * a.ZS)), dim3(NT), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

}  // namespace

// Stride-2, padding-1 3x3x3 convolution with CIN <= 4 input channels and 16 or 32 output channels,
// input [N][CIN][2 Do][2 Ho][2 Wo], output [N][MOUT][Do][Ho][Wo], K = [MOUT / 2][CIN][27][2] (file header).
int tb_conv3d_s2_fewin_f32(const float* in, const float* K, const float* bias, float* out, int N, int Cin, int Mout,
                           int Do, int Ho, int Wo, void* stream) {
  if (!in || !K || !out || N < 1 || Do < 1 || Ho < 1 || Wo < 1) return TB_ERR_INVALID_ARG;
  if (Cin < 1 || Cin > 4 || (Mout != 16 && Mout != 32) || 3 * Wo > 256 || (2 * Wo) % 4 != 0 || 2 * Wo > 256 ||
      (reinterpret_cast<uintptr_t>(in) & 15) != 0)
    return TB_ERR_UNSUPPORTED_SIZE;
  constexpr int TY = 3;
  S2Args a{};
  a.in = in, a.K = K, a.bias = bias, a.out = out;
  a.Do = Do, a.Ho = Ho, a.Wo = Wo, a.Di = 2 * Do, a.Hi = 2 * Ho, a.Wi = 2 * Wo;
  const bool wide = a.Wi > 160;
  a.PX = 4 * (wide ? 64 : 40) + 12;  // = the kernel's compile-time pitch: data at column 4 .. Wi + 3
  a.RR = 2 * TY + 1;
  a.nyb = (Ho + TY - 1) / TY;
  const size_t lds = (size_t)4 * 3 * Cin * a.RR * a.PX;
  if (lds > 163840) return TB_ERR_UNSUPPORTED_SIZE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define TB_S2(CI, MO)                                                                                  \
  if (Cin == CI && Mout == MO) return wide ? launch_s2<CI, MO, 64>(a, lds, N, st) : launch_s2<CI, MO, 40>(a, lds, N, st);
  TB_S2(1, 16) TB_S2(2, 16) TB_S2(3, 16) TB_S2(4, 16) TB_S2(1, 32) TB_S2(2, 32) TB_S2(3, 32) TB_S2(4, 32)
#undef TB_S2
  return TB_ERR_UNSUPPORTED_SIZE;
}

// ConvTranspose3d(Cin -> Mout <= 4, kernel 3, stride 2, padding 1, output_padding 1): x [N][Cin][Di][Hi][Wi]
// -> y [N][Mout][2 Di][2 Hi][2 Wi], W = [Cin][Mout][27] (the module's layout), Cin <= 32.
int tb_convT3d_fewout_f32(const float* x, const float* W, const float* bias, float* y, int N, int Cin, int Mout, int Di,
                          int Hi, int Wi, void* stream) {
  if (!x || !W || !y || N < 1 || Di < 1 || Hi < 1 || Wi < 1) return TB_ERR_INVALID_ARG;
  if (Cin < 1 || Cin > 32 || Mout < 1 || Mout > 4 || Wi % 4 != 0 || Wi > 128 || (reinterpret_cast<uintptr_t>(x) & 15) != 0)
    return TB_ERR_UNSUPPORTED_SIZE;
  // 512 threads over 6 input rows where the two-slot ring of 7 rows fits (one block of 8 waves per CU,
  // two per SIMD, so the scalar weight loads of one wave hide under the other's FMAs); else 256 threads
  const bool big = Wi <= 80 && (size_t)4 * 2 * Cin * 7 * (4 * 20 + 8) <= 163840;
  const int TY = big ? 6 : 256 / Wi >= 3 ? 3 : 256 / Wi >= 2 ? 2 : 1;
  const int nth = big ? 512 : 256;
  TArgs a{};
  a.x = x, a.W = W, a.bias = bias, a.y = y;
  a.Cin = Cin, a.Di = Di, a.Hi = Hi, a.Wi = Wi;
  a.PX = 4 * (Wi <= 80 ? 20 : 32) + 8;  // = the kernel's compile-time pitch
  a.CS = (TY + 1) * a.PX;
  a.nyb = (Hi + TY - 1) / TY;
  const size_t lds = (size_t)4 * 2 * Cin * a.CS;
  if (lds > 163840) return TB_ERR_UNSUPPORTED_SIZE;
  const int per_cu = lds <= 81920 ? 2 : 1;
  a.zlen = zseg(Di, N * a.nyb, per_cu, 1);
  a.ZS = (Di + a.zlen - 1) / a.zlen;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)(N * a.nyb * a.ZS));
  void (*kern)(TArgs) = nullptr;
#define TB_T(MO, T)                                                                    \
  if (Mout == MO && TY == T) kern = Wi <= 80 ? k_convT_fewout<MO, T, 20> : k_convT_fewout<MO, T, 32>;
  TB_T(1, 1) TB_T(1, 2) TB_T(1, 3) TB_T(2, 1) TB_T(2, 2) TB_T(2, 3) TB_T(3, 1) TB_T(3, 2) TB_T(3, 3) TB_T(4, 1)
  TB_T(4, 2) TB_T(4, 3)
#undef TB_T
  // (channels per FMA-loop iteration of the 512-thread form: 1 / 2 / 4 = 296 / 294 / 311 us for the C3
  // 32 -> 3 layer: one)
  constexpr int U = 1;
  if (big && Mout == 3)
    kern = U == 4 ? k_convT_fewout<3, 6, 20, 512, 4> : U == 2 ? k_convT_fewout<3, 6, 20, 512, 2>
                                                      : k_convT_fewout<3, 6, 20, 512>;
  else if (big)
    kern = Mout == 1 ? k_convT_fewout<1, 6, 20, 512> : Mout == 2 ? k_convT_fewout<2, 6, 20, 512>
                                                     : k_convT_fewout<4, 6, 20, 512>;
  if (!kern) return TB_ERR_UNSUPPORTED_SIZE;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, grid, dim3(nth), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

// ------------------------------------------------- stride-1 3x3x3 conv, 16 -> 16 channels, on MFMA
// out[m][p] = b[m] + sum_{c, t} W[m][c][t] X[c][p + t - 1] (padding 1) as Out(16 m x 16 x) =
// W(16 m x 432 k) . X(432 k x 16 x) on mfma_f32_16x16x4f32, k = (tap, channel quad): the block's whole
// W lives in 108 A-fragment registers per lane for the kernel's life; B fragments are LDS reads of the
// staged input planes (lane = (x, channel within the quad): bank-distinct at a channel pitch of 16 mod 32).
// The block marches its (n, YB output rows, z segment) along z with a 3-slot plane ring (the next plane
// in registers, stored over the slot the previous step read last); each wave takes output tiles (row, 16 columns) two at a time (two accumulator chains
// sharing every A fragment).  The input gradient of the same layer is this kernel with
// W'[c][m][t] = W[m][c][26 - t].  Serves the 16-channel full-resolution units (120 x 120 x 80 at C3).
namespace {
struct F16Args {
  const float* x;
  const float* W;     // [16 m][16 c][27]
  const float* bias;  // [16] or null
  const float* add;   // [N][16][D][H][W] summed into y, or null
  float* y;
  int D, H, Wd;
  int ZS, zlen, nyb;
  int PX, RX;  // row pitch (data at column x + 4), channel pitch (= 16 mod 32)
  int flip;    // 1: W is the layer's weight and the call its input gradient: A = W[c][m][26 - t]
  int persist, ncol;  // k_conv3d_fwd16: persistent shares of the ncol = N nyb columns' steps
  int64_t addsn;      // floats between samples of `add` (0: 16 D H W, contiguous)
};

// NS: plane-ring slots.  3: a step's MFMAs read planes z - 1 .. z + 1, plane z + 2 goes over plane z - 1's
// slot after a barrier; 4 (when it fits): plane z + 2 goes into the slot plane z - 2 held, which no wave
// reads in step z -- one barrier per step instead of two.
template <int YB, int NXT, int NTH, bool ADD = false, bool PF = false, int NS = 3>  // output rows per block;
__global__ __launch_bounds__(NTH) void k_conv3d_fwd16(F16Args a) {  // 16-column tiles per row (W = 16 NXT);
                                            // threads; `add` summed into the store; PF: B reads a tap ahead
  constexpr int NWV = NTH / 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NR = YB + 2, W4 = 4 * NXT;  // staged rows; float4 per row
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int D = a.D, H = a.H, Wd = a.Wd, PX = a.PX, RX = a.RX, SS = 16 * RX;
  float* ring = smem;  // [NS][16 c][NR][PX]
  for (int i = tid; i < NS * SS; i += NTH) ring[i] = 0.f;
  // A fragments: lane (m = l & 15, ks = l >> 4); k-step kk = 4 t + cq covers channel 4 cq + ks at tap t
  const int li = lane & 15, ks = lane >> 4;
  float af[108];
#pragma unroll
  for (int kk = 0; kk < 108; ++kk) {
    const int c = 4 * (kk & 3) + ks, t = kk >> 2;
    af[kk] = a.flip ? a.W[(c * 16 + li) * 27 + 26 - t] : a.W[(li * 16 + c) * 27 + t];
  }
  const float bm[4] = {a.bias ? a.bias[4 * ks] : 0.f, a.bias ? a.bias[4 * ks + 1] : 0.f,
                       a.bias ? a.bias[4 * ks + 2] : 0.f, a.bias ? a.bias[4 * ks + 3] : 0.f};
  // the block's steps: (n, row block, plane) linearised as column (n, yb) major, plane minor.  a.persist: a
  // contiguous 1/gridDim share of all of them (one block per CU, every CU busy, a share spans at most a
  // few columns, each marched on its own); else the (n, yb, z segment) of blockIdx
  int64_t s_beg, s_end;
  if (a.persist) {
    const int64_t T = (int64_t)a.ncol * D;
    s_beg = T * blockIdx.x / gridDim.x, s_end = T * (blockIdx.x + 1) / gridDim.x;
  } else {
    int b = (int)blockIdx.x;
    const int zs = b % a.ZS;
    b /= a.ZS;
    const int zb = zs * a.zlen;
    s_beg = (int64_t)b * D + zb, s_end = (int64_t)b * D + min(D, zb + a.zlen);
  }
  for (int64_t sg = s_beg; sg < s_end;) {
  const int col = (int)(sg / D), z0 = (int)(sg - (int64_t)col * D);
  const int z1 = (int)min((int64_t)D, z0 + (s_end - sg));
  sg += z1 - z0;
  const int yb = col % a.nyb, n = col / a.nyb;
  const int y0 = yb * YB;
  const int64_t plane = (int64_t)H * Wd, plane4 = plane / 4;
  const float4* xb = reinterpret_cast<const float4*>(a.x + (int64_t)n * 16 * D * plane);
  constexpr int NL = (16 * NR * W4 + NTH - 1) / NTH;
  int gof[NL], lof[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + NTH * j;
    const int q = i % W4, t = i / W4, r = t % NR, c = t / NR;
    const int yi = y0 - 1 + r;
    const bool ok = i < 16 * NR * W4 && yi >= 0 && yi < H;
    gof[j] = ok ? (int)((int64_t)c * D * plane4 + ((int64_t)yi * Wd + 4 * q) / 4) : -1;
    // rows outside the volume store zeros over their (zero) staging rows; slots past the staged block
    // store zeros over the first four pad columns -- every lane stores, so that no path skips the wait for
    // the plane loads (a skippable wait makes the compiler wait again, for the output stores too, before
    // the next plane's loads reuse the registers)
    lof[j] = i < 16 * NR * W4 ? c * RX + r * PX + 4 + 4 * q : 0;
  }
  float4 rg[NL];
  auto load = [&](int zi) {
    const bool in = zi >= 0 && zi < D;
    const float4* src = xb + (int64_t)(in ? zi : 0) * plane4;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      rg[j] = src[gof[j] < 0 ? 0 : gof[j]];  // zeroed at the store (a select here waits for the load)
    }
  };
  auto store = [&](int zi) {
    float* d = ring + ((zi + NS) % NS) * SS;
    const bool in = zi >= 0 && zi < D;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      *reinterpret_cast<float4*>(d + lof[j]) = in && gof[j] >= 0 ? rg[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  __syncthreads();
  load(z0 - 1);
  store(z0 - 1);
  load(z0);
  store(z0);
  load(z0 + 1);
  store(z0 + 1);
  // every start-up load (A fragments, bias, the first planes) retired here, so that the compiler does not
  // wait for the loop's plane loads (vmcnt(0)) before a step's first MFMA
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  // B lane base: channel 4 cq + ks (cq added per k-step), column x = li of the tile (+ tx - 1 at + 4)
  const int bl = ks * RX + li + 3;
  const int64_t oplane = plane;
  float* yb0 = a.y + (int64_t)n * 16 * D * oplane;
  const float* ab0 = ADD ? a.add + (int64_t)n * (a.addsn ? a.addsn : 16 * D * oplane) : nullptr;
  constexpr int NT = YB * NXT;                        // tiles per step
  constexpr int NIT = (NT + 2 * NWV - 1) / (2 * NWV);  // tile pairs per wave
  // step z: fetch plane z + 2 (registers) | MFMAs over planes z - 1 .. z + 1 | barrier | plane z + 2 into
  // the slot plane z - 1 held | the step's output stores | barrier.  The output stores come after the
  // plane's LDS store, so the wait for the plane loads never includes an output store's write-back.
  for (int z = z0; z < z1; ++z) {
    const bool more = z + 1 < z1;
    if (more) load(z + 2);
    // ADD: the step's `add` values fetched now, summed at the stores after the MFMAs (loaded at the store
    // they would be waited for there)
    float av[NIT][2][4];
    if constexpr (ADD) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int t0 = wave + 2 * NWV * it;
        if (t0 >= NT) break;
        const int t1 = t0 + NWV < NT ? t0 + NWV : t0;
        const int yy0 = t0 / NXT, x00 = 16 * (t0 - yy0 * NXT);
        const int yy1 = t1 / NXT, x01 = 16 * (t1 - yy1 * NXT);
        const int ya = min(y0 + yy0, H - 1), yc = min(y0 + yy1, H - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 4 * ks + r;
          av[it][0][r] = ab0[((int64_t)m * D + z) * oplane + (int64_t)ya * Wd + x00 + li];
          av[it][1][r] = ab0[((int64_t)m * D + z) * oplane + (int64_t)yc * Wd + x01 + li];
        }
      }
    }
    const float* s0 = ring + ((z + NS - 1) % NS) * SS + bl;  // tz = 0: plane z - 1
    const float* s1 = ring + (z % NS) * SS + bl;
    const float* s2 = ring + ((z + 1) % NS) * SS + bl;
    f32x4 acc[NIT][2];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {  // tiles t0 and t0 + NWV of this wave
      const int t0 = wave + 2 * NWV * it;
      if (t0 >= NT) break;
      const int t1 = t0 + NWV < NT ? t0 + NWV : t0;
      const int yy0 = t0 / NXT, x00 = 16 * (t0 - yy0 * NXT);
      const int yy1 = t1 / NXT, x01 = 16 * (t1 - yy1 * NXT);
      const int o0 = yy0 * PX + x00, o1 = yy1 * PX + x01;
      f32x4 acc0 = {bm[0], bm[1], bm[2], bm[3]}, acc1 = acc0;
      if constexpr (PF) {  // the next tap's 8 B fragments read while this tap's 8 MFMAs run
        float bq[2][8];
        auto ldb = [&](int t, float (&q)[8]) {
          const int tz = t / 9, ty = (t / 3) % 3, tx = t % 3;
          const float* sl = tz == 0 ? s0 : tz == 1 ? s1 : s2;
#pragma unroll
          for (int cq = 0; cq < 4; ++cq) {
            const int off = 4 * cq * RX + ty * PX + tx;
            q[2 * cq] = sl[o0 + off], q[2 * cq + 1] = sl[o1 + off];
          }
        };
        ldb(0, bq[0]);
#pragma unroll
        for (int t = 0; t < 27; ++t) {
          if (t + 1 < 27) ldb(t + 1, bq[(t + 1) & 1]);
#pragma unroll
          for (int cq = 0; cq < 4; ++cq) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[4 * t + cq], bq[t & 1][2 * cq], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[4 * t + cq], bq[t & 1][2 * cq + 1], acc1, 0, 0, 0);
          }
        }
        // schedule: one MFMA, then one LDS read (the next tap's), alternating
#pragma unroll
        for (int i = 0; i < 216; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      } else {
#pragma unroll
      for (int tz = 0; tz < 3; ++tz) {
        const float* sl = tz == 0 ? s0 : tz == 1 ? s1 : s2;
#pragma unroll
        for (int ty = 0; ty < 3; ++ty)
#pragma unroll
          for (int tx = 0; tx < 3; ++tx) {
            const int t = tz * 9 + ty * 3 + tx;
#pragma unroll
            for (int cq = 0; cq < 4; ++cq) {
              const int off = 4 * cq * RX + ty * PX + tx;
              const float b0 = sl[o0 + off], b1 = sl[o1 + off];
              acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[4 * t + cq], b0, acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[4 * t + cq], b1, acc1, 0, 0, 0);
            }
          }
      }
      }
      acc[it][0] = acc0, acc[it][1] = acc1;
    }
    if constexpr (NS == 3) __syncthreads();
    store(z + 2);  // unconditionally (after the last step a dead slot): no path skips the loads' wait
#pragma unroll
    for (int it = 0; it < NIT; ++it) {  // C: column x = li, rows m = 4 ks + r
      const int t0 = wave + 2 * NWV * it;
      if (t0 >= NT) break;
      const int t1 = t0 + NWV < NT ? t0 + NWV : t0;
      const int yy0 = t0 / NXT, x00 = 16 * (t0 - yy0 * NXT);
      const int yy1 = t1 / NXT, x01 = 16 * (t1 - yy1 * NXT);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * ks + r;
        const int64_t o0 = ((int64_t)m * D + z) * oplane + (int64_t)(y0 + yy0) * Wd + x00 + li;
        const int64_t o1 = ((int64_t)m * D + z) * oplane + (int64_t)(y0 + yy1) * Wd + x01 + li;
        if (y0 + yy0 < H) yb0[o0] = ADD ? acc[it][0][r] + av[it][0][r] : acc[it][0][r];
        if (t1 != t0 && y0 + yy1 < H) yb0[o1] = ADD ? acc[it][1][r] + av[it][1][r] : acc[it][1][r];
      }
    }
    __syncthreads();
  }
  }
}
}  // namespace

// (Round 6: the DMA-staged plane variant (439 vs 382 us) and the split-precision bf16 variant
// k_conv16_x3 (no gain in the step) were measured, rejected and removed; DESIGN.md records them.)


// Conv3d(16 -> 16, 3, stride 1, padding 1) forward: x [N][16][D][H][W] -> y [N][16][D][H][W], W % 16 == 0,
// W <= 128; weight [16][16][27], bias [16] or NULL.  (csrc/conv_up.hip, k_conv3d_fwd16)
int tb_conv3d_fwd16_f32(const float* x, const float* W, const float* bias, float* y, int N, int D, int H, int Wd,
                        void* stream) {
  return tb_conv3d_fwd16_add_f32(x, W, bias, nullptr, y, N, D, H, Wd, stream);
}

static int fwd16_call(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int D, int H,
                      int Wd, int flip, void* stream, int64_t add_sn = 0);

int tb_conv3d_fwd16_add_f32(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int D,
                            int H, int Wd, void* stream) {
  return fwd16_call(x, W, bias, add, y, N, D, H, Wd, 0, stream);
}

int tb_conv3d_fwd16_dgrad_f32(const float* gy, const float* W, const float* add, int64_t add_sn, float* dx, int N, int D,
                              int H, int Wd, void* stream) {
  return fwd16_call(gy, W, nullptr, add, dx, N, D, H, Wd, 1, stream, add_sn);
}

static int fwd16_call(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int D, int H,
                      int Wd, int flip, void* stream, int64_t add_sn) {
  if (!x || !W || !y || N < 1 || D < 1 || H < 1 || Wd < 1) return TB_ERR_INVALID_ARG;
  if (Wd % 16 != 0 || Wd > 128 || (reinterpret_cast<uintptr_t>(x) & 15) != 0) return TB_ERR_UNSUPPORTED_SIZE;
  // output rows per block (C3, W = 80: YB 2 / 3 / 4 = 478 / 419 / 482 us -- the YB x 5 tiles of a step
  // over 4 waves x 2 chains: 10 of 16, 15 of 16, 20 of 24 slots used; YB = 2's second block per CU did not
  // make up for it): only YB = 3 is instantiated
  constexpr int YB = 3;
  F16Args a{};
  a.x = x, a.W = W, a.bias = bias, a.add = add, a.y = y, a.D = D, a.H = H, a.Wd = Wd;
  a.flip = flip;
  a.addsn = add_sn;
  a.PX = Wd + 8;
  a.RX = (YB + 2) * a.PX;
  while ((a.RX & 31) != 16) ++a.RX;
  a.nyb = (H + YB - 1) / YB;
  const int NS = (size_t)4 * 4 * 16 * a.RX <= 163840 ? 4 : 3;  // 4-slot plane ring where it fits
  const size_t lds = (size_t)NS * 4 * 16 * a.RX;
  if (lds > 163840) return TB_ERR_UNSUPPORTED_SIZE;
  const int per_cu = 163840 / (int)lds >= 2 ? 2 : 1;
  a.zlen = zseg(D, N * a.nyb, per_cu, 2);
  a.ZS = (D + a.zlen - 1) / a.zlen;
  void (*kern)(F16Args) = nullptr;
  // 512 threads per block: 8 waves, 2 per SIMD sharing the matrix core, hide the B-fragment LDS reads the
  // compiler issues only 1-3 ahead (YB = 3: 421 -> 365 us per C3 call against 256 threads)
  constexpr int NTv = 512;
  // the B fragments read a tap ahead of their MFMAs, interleaved one LDS read per MFMA (sched_group_barrier)
  // and a 4-slot plane ring, one barrier per step (C3, by scripts/diag/conv_kern_bench.py: forward
  // 385 -> 374 us, input gradient 361 -> 353 us against the earlier form, still the fallback below)
  constexpr bool PFv = true;
  if (PFv && YB == 3 && NTv == 512 && Wd == 80) {
    kern = add ? (NS == 4 ? k_conv3d_fwd16<3, 5, 512, true, true, 4> : k_conv3d_fwd16<3, 5, 512, true, true, 3>)
               : (NS == 4 ? k_conv3d_fwd16<3, 5, 512, false, true, 4> : k_conv3d_fwd16<3, 5, 512, false, true, 3>);
  } else
#define TB_F16C(Y, X, T) \
  kern = add ? (NS == 4 ? k_conv3d_fwd16<Y, X, T, true, false, 4> : k_conv3d_fwd16<Y, X, T, true, false, 3>) \
             : (NS == 4 ? k_conv3d_fwd16<Y, X, T, false, false, 4> : k_conv3d_fwd16<Y, X, T, false, false, 3>);
#define TB_F16(Y, T)                                                                                   \
  if (YB == Y && NTv == T) switch (Wd / 16) {                                                          \
      case 1: TB_F16C(Y, 1, T) break;                                                                  \
      case 2: TB_F16C(Y, 2, T) break;                                                                  \
      case 3: TB_F16C(Y, 3, T) break;                                                                  \
      case 4: TB_F16C(Y, 4, T) break;                                                                  \
      case 5: TB_F16C(Y, 5, T) break;                                                                  \
      case 6: TB_F16C(Y, 6, T) break;                                                                  \
      case 7: TB_F16C(Y, 7, T) break;                                                                  \
      case 8: TB_F16C(Y, 8, T) break;                                                                  \
      default: return TB_ERR_UNSUPPORTED_SIZE;                                                         \
    }
  TB_F16(3, 512)
#undef TB_F16
#undef TB_F16C
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  // persistent shares when the (n, yb, z segment) grid leaves CUs idle (C3: 240 blocks of 256)
  constexpr int persist_env = 1;
  a.ncol = N * a.nyb;
  unsigned nblk = (unsigned)(N * a.nyb * a.ZS);
  a.persist = persist_env && per_cu == 1 && (int64_t)a.ncol * D >= 8LL * ncu_count() && nblk % ncu_count() != 0;
  if (a.persist) nblk = (unsigned)ncu_count();
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(NTv), lds, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

// ------------------------------------------------- ConvTranspose3d(64 -> 16, 3, s2, p1, op1) on MFMA
// Sub-pixel form (as k_convT_fewout): input position i = (z, y, x) gives the 8 outputs 2 i + p, p in
// {0, 1}^3; per axis parity 0 takes tap 1 at offset 0, parity 1 takes tap 2 at offset 0 and tap 0 at
// offset +1, so the 27 taps split over the 8 parities and each is a real multiply-add.  As products:
// Out_p(16 m x 16 positions) = sum over p's taps and the 64 channels of W[c][m][t] X[c][i + delta(t)],
// on mfma_f32_16x16x4f32 with k = (tap, channel quad).  Wave g holds the A fragments of channel group
// g (channels 16 g .. 16 g + 15: 108 registers) and accumulates all 8 parities of a 16-position tile
// (positions = flattened (row, column) of the block's YB input rows); the four groups' partial tiles
// meet in LDS (double-buffered, one barrier per tile), where wave w sums parities (w >> 1, w & 1, 0 / 1)
// and writes them as (px = 0, 1) float2 pairs.  The block marches (n, YB rows, z segment) along z with
// a 2-slot input plane ring (plane z and z + 1; the next plane in registers).  Replaces MIOpen's
// col2im GEMM pair for the U-Net's up1 ConvTranspose3d (64 -> 16, 60 x 60 x 40 -> 120 x 120 x 80 at C3).
namespace {
struct T64Args {
  const float* x;     // [N][64][Di][Hi][Wi]
  const float* W;     // [64 c][16 m][27]
  const float* bias;  // [16] or null
  float* y;           // [N][16][2 Di][2 Hi][2 Wi]
  int Di, Hi, Wi;
  int ZS, zlen, nyb;
  int PX, RX;         // staged row pitch (data at columns 0 .. Wi - 1, zeros after), channel pitch (16 mod 32)
};

// G channel groups (Cin = 16 G): with G = 2 the waves (g, h) also split the position tiles (h = tile parity).
template <int G, int YB, int NL>  // NL: float4 staging pieces per thread (Cin (YB + 1) Wi / 4 <= 256 NL)
__global__ __launch_bounds__(256) void k_convT_mfma64(T64Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NR = YB + 1;  // staged rows: y0 .. y0 + YB
  constexpr int CIN = 16 * G, HT = 4 / G;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w % G, h = w / G;  // channel group, tile phase of this wave
  const int Di = a.Di, Hi = a.Hi, Wi = a.Wi, PX = a.PX, RX = a.RX, SS = CIN * RX;
  float* ring = smem;                   // [2][Cin][NR][PX]
  float* part = smem + 2 * SS;          // [2 buf][4 waves][8 parities][16 m][16 pos]
  for (int i = tid; i < 2 * SS; i += 256) ring[i] = 0.f;
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int y0 = yb * YB;
  const int z0 = zs * a.zlen, z1 = min(Di, z0 + a.zlen);
  const int li = lane & 15, ks = lane >> 4;
  float af[108];  // k-step 4 t + cq: channel 16 g + 4 cq + ks, tap t, output channel li
#pragma unroll
  for (int kk = 0; kk < 108; ++kk) af[kk] = a.W[((16 * g + 4 * (kk & 3) + ks) * 16 + li) * 27 + (kk >> 2)];
  const int64_t plane = (int64_t)Hi * Wi;
  const float* xb = a.x + (int64_t)n * CIN * Di * plane;
  // staging: float4 pieces of (channel, row, column quad); Wi % 4 == 0.  gof: offset in the
  // channel-plane's floats (-1: a row past Hi, staged as zeros), lof: LDS offset
  const int W4 = Wi >> 2, per_c = NR * W4, total = CIN * per_c;
  const int64_t cstride = (int64_t)Di * plane;
  int gof[NL], lof[NL], gch[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + 256 * j;
    const int c = i / per_c, r2 = i - c * per_c, r = r2 / W4, q = r2 - r * W4;
    const int yi = y0 + r;
    lof[j] = i < total ? c * RX + r * PX + 4 * q : Wi;  // past the block: zeros over row 0's pad columns
    gof[j] = (i < total && yi < Hi) ? yi * Wi + 4 * q : -1;
    gch[j] = i < total ? c : 0;
  }
  float4 rg[NL];
  auto load = [&](int zi) {
    const bool in = zi < Di;
    const float* src = xb + (int64_t)(in ? zi : 0) * plane;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const bool ok = in && gof[j] >= 0;  // zeroed at the store (a select here waits for the load)
      rg[j] = *reinterpret_cast<const float4*>(src + gch[j] * cstride + (ok ? gof[j] : 0));
    }
  };
  auto store = [&](int zi) {  // every lane stores (see k_conv3d_fwd16: no path skips the loads' wait)
    float* d = ring + (zi & 1) * SS;
    const bool in = zi < Di;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      *reinterpret_cast<float4*>(d + lof[j]) = (in && gof[j] >= 0) ? rg[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float bm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bm[r] = a.bias ? a.bias[4 * ks + r] : 0.f;
  __syncthreads();
  load(z0);
  store(z0);
  load(z0 + 1);
  store(z0 + 1);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // start-up loads retired (as in k_conv3d_fwd16)
  __syncthreads();
  const int npos = YB * Wi, ntile = (npos + 15) / 16;
  const int64_t oplane = 4 * plane, orow = 2 * Wi;
  float* yb0 = a.y + (int64_t)n * 16 * (2 * Di) * oplane;
  // (tile phase h', parity pair (pz, py, 0 / 1)) combos over the waves: the G groups' partials summed
  auto sums = [&](int z, int t0, int pb) {
    const float* pr = part + pb * 4 * 8 * 256;
    for (int k = w; k < 4 * HT; k += 4) {
      const int hq = k >> 2, pz = (k >> 1) & 1, py = k & 1, q0 = pz * 4 + py * 2;
      const int pq = 16 * (t0 + hq) + li, yq = pq / Wi, xq = pq - yq * Wi;
      const bool okp = t0 + hq < ntile && pq < npos && y0 + yq < Hi;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * ks + r, e = m * 16 + li;
        float v0 = bm[r], v1 = bm[r];
#pragma unroll
        for (int v = 0; v < G; ++v) {
          v0 += pr[((hq * G + v) * 8 + q0) * 256 + e];
          v1 += pr[((hq * G + v) * 8 + q0 + 1) * 256 + e];
        }
        if (okp)
          *reinterpret_cast<float2*>(yb0 + ((int64_t)m * (2 * Di) + 2 * z + pz) * oplane +
                                     (int64_t)(2 * (y0 + yq) + py) * orow + 2 * xq) = make_float2(v0, v1);
      }
    }
  };
  int buf = 0;
  // step z: fetch plane z + 2 | per tile: MFMAs, partials, barrier, the previous tile's sums and stores |
  // plane z + 2 over plane z's slot | the last tile's sums and stores | barrier.  The plane's LDS store
  // waits for its loads and the stores of all but the last tile (issued a tile earlier), never for the
  // stores just issued.
  for (int z = z0; z < z1; ++z) {
    if (z + 1 < z1) load(z + 2);
    const float* sz[2] = {ring + (z & 1) * SS, ring + ((z + 1) & 1) * SS};
    for (int t0 = 0; t0 < ntile; t0 += HT) {
      const int tI = t0 + h;
      const int p = 16 * tI + li, pc = p < npos ? p : npos - 1;
      const int yy = pc / Wi, xx = pc - yy * Wi;
      const int bl = (16 * g + ks) * RX + yy * PX + xx;
      f32x4 acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tz = 0; tz < 3; ++tz)
#pragma unroll
        for (int ty = 0; ty < 3; ++ty)
#pragma unroll
          for (int tx = 0; tx < 3; ++tx) {
            const int t = tz * 9 + ty * 3 + tx;
            const int par = (tz != 1) * 4 + (ty != 1) * 2 + (tx != 1);
            const float* s = sz[tz == 0] + bl + (ty == 0) * PX + (tx == 0);
#pragma unroll
            for (int cq = 0; cq < 4; ++cq)
              acc[par] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[4 * t + cq], s[4 * cq * RX], acc[par], 0, 0, 0);
          }
      // partial tiles: C layout column = position li, rows m = 4 ks + r
      float* pw = part + (buf * 4 + w) * 8 * 256;
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[q * 256 + (4 * ks + r) * 16 + li] = acc[q][r];
      __syncthreads();
      if (t0 > 0) sums(z, t0 - HT, buf ^ 1);
      buf ^= 1;
    }
    store(z + 2);  // slot (z + 2) & 1 = plane z's, read by no wave after the last tile's barrier; unconditional
    sums(z, ((ntile - 1) / HT) * HT, buf ^ 1);
    __syncthreads();
  }
}
}  // namespace

// ConvTranspose3d(64 -> 16, 3, stride 2, padding 1, output_padding 1) forward:
// x [N][64][Di][Hi][Wi] -> y [N][16][2Di][2Hi][2Wi]; weight [64][16][3][3][3] as the module holds it,
// bias [16] or NULL; Wi % 4 == 0, Wi <= 64.  (csrc/conv_up.hip, k_convT_mfma64)
int tb_convT3d_mfma64_f32(const float* x, const float* W, const float* bias, float* y, int N, int Di, int Hi, int Wi,
                          void* stream) {
  return tb_convT3d_mfma_f32(x, W, bias, y, N, 64, Di, Hi, Wi, stream);
}

// ConvTranspose3d(Cin -> 16, 3, s2, p1, op1) forward for Cin = 32 or 64 (also the input gradient of
// Conv3d(16 -> Cin, s2, p1) with that layer's weight); as tb_convT3d_mfma64_f32 otherwise.
int tb_convT3d_mfma_f32(const float* x, const float* W, const float* bias, float* y, int N, int Cin, int Di, int Hi,
                        int Wi, void* stream) {
  if (!x || !W || !y || N < 1 || Di < 1 || Hi < 1 || Wi < 1) return TB_ERR_INVALID_ARG;
  if (Cin != 32 && Cin != 64) return TB_ERR_UNSUPPORTED_SIZE;
  if (Wi % 4 != 0 || Wi > 64 || (reinterpret_cast<uintptr_t>(x) & 15) != 0 || (reinterpret_cast<uintptr_t>(y) & 7) != 0)
    return TB_ERR_UNSUPPORTED_SIZE;
  constexpr int YB = 2;
  T64Args a{};
  a.x = x, a.W = W, a.bias = bias, a.y = y, a.Di = Di, a.Hi = Hi, a.Wi = Wi;
  a.PX = Wi + 4;
  a.RX = (YB + 1) * a.PX;
  while ((a.RX & 31) != 16) ++a.RX;
  a.nyb = (Hi + YB - 1) / YB;
  const size_t lds = (size_t)4 * (2 * Cin * a.RX + 2 * 4 * 8 * 256);
  if (lds > 163840) return TB_ERR_UNSUPPORTED_SIZE;
  a.zlen = zseg(Di, N * a.nyb, 1, 1);
  a.ZS = (Di + a.zlen - 1) / a.zlen;
  const int nl = (Cin * (YB + 1) * (Wi / 4) + 255) / 256;
  void (*kern)(T64Args) = nullptr;
  switch (nl) {
#define TB_NL(k) \
  case k: kern = Cin == 64 ? k_convT_mfma64<4, YB, k> : k_convT_mfma64<2, YB, k>; break;
    TB_NL(1) TB_NL(2) TB_NL(3) TB_NL(4) TB_NL(5) TB_NL(6) TB_NL(7) TB_NL(8) TB_NL(9) TB_NL(10) TB_NL(11) TB_NL(12)
#undef TB_NL
    default: return TB_ERR_UNSUPPORTED_SIZE;
  }
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, dim3((unsigned)(N * a.nyb * a.ZS)), dim3(256), lds, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}

// ------------------------------------------------- stride-1 3x3x3 conv, C -> C channels (C = 32, 64), on MFMA
// The k_conv3d_fwd16 product with the input channels split over the block's waves: wave w holds the A
// fragments (108 registers) of channel group g = w % G (16 channels) for output tile m = w / G of the
// block's 4 / G; it accumulates NC position tiles at once (NC independent chains; positions = the
// flattened (row, column) of the block's YB rows, so rows need not be a multiple of 16) and the G
// groups' partial tiles meet in LDS, where the waves sum them and store.  A 3-slot plane ring as in
// k_conv3d_fwd16.  The input gradient of the same layer is this kernel with W'[c][m][t] = W[m][c][26 - t].
// Serves the U-Net's 32- and 64-channel units (60 x 60 x 40 and 30 x 30 x 20 at C3).
namespace {
struct S1Args {
  const float* x;     // [N][C][D][H][W]
  const float* W;     // [C m][C c][27]
  const float* bias;  // [C] or null
  const float* add;   // summed into y (y's layout), or null
  float* y;
  int D, H, Wd, YB;
  int ZS, zlen, nyb, MG;  // z segments, row blocks, output-tile groups
  int PX, RX;             // row pitch (data at column x + 4), channel pitch (16 mod 32)
  int flip;               // 1: W is the layer's weight and the call its input gradient (W[c][m][26 - t])
  int64_t addsn;          // floats between samples of `add` (0: contiguous)
};

template <int G, int NC, int NL, int NTH, bool ADD = false>  // NTH 512: two waves per role, alternate tiles
__global__ __launch_bounds__(NTH) void k_conv3d_mfma_s1(S1Args a) {  // (NWG phases); `add` summed into the store
  constexpr int CIN = 16 * G, MTB = 4 / G, NWG = NTH / 256;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w % G, mt = (w / G) % MTB, h = w / 4;
  const int D = a.D, H = a.H, Wd = a.Wd, YB = a.YB, PX = a.PX, RX = a.RX, SS = CIN * RX;
  const int NR = YB + 2;
  float* ring = smem;            // [3][CIN][NR rows][PX]
  float* part = smem + 3 * SS;   // [NTH / 64 waves][NC][16 m][16 pos]
  float* bsm = part + (NTH / 64) * NC * 256;  // the block's bias values [MTB * 16] (no global load in the loop)
  for (int i = tid; i < 3 * SS; i += NTH) ring[i] = 0.f;
  int b = (int)blockIdx.x;
  const int zs = b % a.ZS;
  b /= a.ZS;
  const int mg = b % a.MG;
  b /= a.MG;
  const int yb = b % a.nyb, n = b / a.nyb;
  const int COUT = 16 * MTB * a.MG;
  const int y0 = yb * YB;
  const int z0 = zs * a.zlen, z1 = min(D, z0 + a.zlen);
  const int li = lane & 15, ks = lane >> 4;
  const int m0 = (mg * MTB + mt) * 16;
  if (tid < MTB * 16) bsm[tid] = a.bias ? a.bias[mg * MTB * 16 + tid] : 0.f;
  float af[108];
#pragma unroll
  for (int kk = 0; kk < 108; ++kk) {
    const int c = 16 * g + 4 * (kk & 3) + ks, t = kk >> 2;
    af[kk] = a.flip ? a.W[(c * CIN + m0 + li) * 27 + 26 - t] : a.W[((m0 + li) * CIN + c) * 27 + t];
  }
  const int64_t plane = (int64_t)H * Wd, cstride = (int64_t)D * plane;
  const float* xb = a.x + (int64_t)n * CIN * cstride;
  const int W4 = Wd >> 2, per_c = NR * W4, total = CIN * per_c;
  int gof[NL], lof[NL], gch[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + NTH * j;
    const int c = i / per_c, r2 = i - c * per_c, r = r2 / W4, q = r2 - r * W4;
    const int yi = y0 - 1 + r;
    lof[j] = i < total ? c * RX + r * PX + 4 + 4 * q : 0;  // past the block: zeros over pad columns 0..3
    gof[j] = (i < total && yi >= 0 && yi < H) ? yi * Wd + 4 * q : -1;
    gch[j] = i < total ? c : 0;
  }
  float4 rg[NL];
  auto load = [&](int zi) {
    const bool in = zi >= 0 && zi < D;
    const float* src = xb + (int64_t)(in ? zi : 0) * plane;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const bool ok = in && gof[j] >= 0;  // zeroed at the store (a select here waits for the load)
      rg[j] = *reinterpret_cast<const float4*>(src + gch[j] * cstride + (ok ? gof[j] : 0));
    }
  };
  auto store = [&](int zi) {  // every lane stores (see k_conv3d_fwd16: no path skips the loads' wait)
    float* d = ring + ((zi + 3) % 3) * SS;
    const bool in = zi >= 0 && zi < D;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      *reinterpret_cast<float4*>(d + lof[j]) = (in && gof[j] >= 0) ? rg[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  __syncthreads();
  load(z0 - 1);
  store(z0 - 1);
  load(z0);
  store(z0);
  load(z0 + 1);
  store(z0 + 1);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // start-up loads retired (as in k_conv3d_fwd16)
  __syncthreads();
  // the host sizes YB so that a step's positions fit the block's NWG x NC chains: one tile round per step
  const int npos = YB * Wd;
  float* ybase = a.y + (int64_t)n * COUT * cstride;
  const float* abase = ADD ? a.add + (int64_t)n * (a.addsn ? a.addsn : COUT * cstride) : nullptr;
  constexpr int NK = (MTB * NWG * NC + NTH / 64 - 1) / (NTH / 64);  // sum-phase combos per wave
  int bl[NC];  // chain c of this wave: position tile NWG c + h
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int p = 16 * (NWG * c + h) + li, pc = p < npos ? p : npos - 1;
    const int yy = pc / Wd, xx = pc - yy * Wd;
    bl[c] = (16 * g + ks) * RX + yy * PX + xx + 3;
  }
  // step z: fetch plane z + 2 | MFMAs over planes z - 1 .. z + 1 into the group partials | barrier | plane
  // z + 2 over plane z - 1's slot, the partials summed and stored | barrier
  for (int z = z0; z < z1; ++z) {
    if (z + 1 < z1) load(z + 2);
    // ADD: the step's `add` values fetched now, summed in the store phase (as in k_conv3d_fwd16)
    float av[NK][4];
    if constexpr (ADD) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const int k = w + kk * (NTH / 64);
        if (k >= MTB * NWG * NC) break;
        const int mq = k / (NWG * NC), r2 = k - mq * (NWG * NC), hq = r2 / NC, c = r2 - hq * NC;
        const int p = 16 * (NWG * c + hq) + li, pc = p < npos ? p : npos - 1;
        const int yy = pc / Wd, xx = pc - yy * Wd, yr = min(y0 + yy, H - 1);
        const int mb = (mg * MTB + mq) * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          av[kk][r] = abase[(int64_t)(mb + 4 * ks + r) * cstride + (int64_t)z * plane + (int64_t)yr * Wd + xx];
      }
    }
    const float* sp[3] = {ring + ((z + 2) % 3) * SS, ring + (z % 3) * SS, ring + ((z + 1) % 3) * SS};
    f32x4 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    // (B reads a k-step ahead with per-step scheduling barriers measured no change, 209 / 120 us)
#pragma unroll
    for (int tz = 0; tz < 3; ++tz)
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          const int t = tz * 9 + ty * 3 + tx;
          const float* s = sp[tz] + ty * PX + tx;
#pragma unroll
          for (int cq = 0; cq < 4; ++cq)
#pragma unroll
            for (int c = 0; c < NC; ++c)
              acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[4 * t + cq], s[bl[c] + 4 * cq * RX], acc[c], 0, 0, 0);
        }
    float* pw = part + w * NC * 256;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) pw[c * 256 + (4 * ks + r) * 16 + li] = acc[c][r];
    __syncthreads();
    store(z + 2);  // unconditionally (after the last step a dead slot)
    // (output tile mt', phase h', chain c) combos over the waves: the G groups' partials summed + bias
    // (k, kk): sum-phase combo k = w + kk * waves; kk indexes the prefetched add values (ADD only: the
    // unrolled form keeps them in registers; the plain form keeps the runtime loop and its register count)
    auto combo = [&](int k, int kk) {
      const int mq = k / (NWG * NC), r2 = k - mq * (NWG * NC), hq = r2 / NC, c = r2 - hq * NC;
      const int p = 16 * (NWG * c + hq) + li;
      const int yy = p / Wd, xx = p - yy * Wd;
      const bool ok = p < npos && y0 + yy < H;
      const int mb = (mg * MTB + mq) * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * ks + r;
        float v = bsm[mq * 16 + m];
#pragma unroll
        for (int gg = 0; gg < G; ++gg) v += part[((hq * 4 + mq * G + gg) * NC + c) * 256 + m * 16 + li];
        const int64_t o = (int64_t)(mb + m) * cstride + (int64_t)z * plane + (int64_t)(y0 + yy) * Wd + xx;
        if (ok) ybase[o] = ADD ? v + av[kk][r] : v;
      }
    };
    if constexpr (ADD) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const int k = w + kk * (NTH / 64);
        if (k >= MTB * NWG * NC) break;
        combo(k, kk);
      }
    } else {
      for (int k = w; k < MTB * NWG * NC; k += NTH / 64) combo(k, 0);
    }
    __syncthreads();
  }
}
}  // namespace

// Conv3d(C -> C, 3, stride 1, padding 1) forward for C = 32 or 64: x [N][C][D][H][W] -> y, W % 4 == 0,
// W <= 64; weight [C][C][27], bias [C] or NULL.  (csrc/conv_up.hip, k_conv3d_mfma_s1)
int tb_conv3d_mfma_f32(const float* x, const float* W, const float* bias, float* y, int N, int C, int D, int H, int Wd,
                       void* stream) {
  return tb_conv3d_mfma_add_f32(x, W, bias, nullptr, y, N, C, D, H, Wd, stream);
}

static int mfma_call(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int C, int D,
                     int H, int Wd, int flip, void* stream, int64_t add_sn = 0);

int tb_conv3d_mfma_add_f32(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int C,
                           int D, int H, int Wd, void* stream) {
  return mfma_call(x, W, bias, add, y, N, C, D, H, Wd, 0, stream);
}

int tb_conv3d_mfma_dgrad_f32(const float* gy, const float* W, const float* add, int64_t add_sn, float* dx, int N, int C,
                             int D, int H, int Wd, void* stream) {
  return mfma_call(gy, W, nullptr, add, dx, N, C, D, H, Wd, 1, stream, add_sn);
}

static int mfma_call(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int C, int D,
                     int H, int Wd, int flip, void* stream, int64_t add_sn) {
  if (!x || !W || !y || N < 1 || D < 1 || H < 1 || Wd < 1) return TB_ERR_INVALID_ARG;
  if ((C != 32 && C != 64) || Wd % 4 != 0 || Wd > 64 || (reinterpret_cast<uintptr_t>(x) & 15) != 0)
    return TB_ERR_UNSUPPORTED_SIZE;
  // 4 waves with 5 chains each (8 waves, two per role on alternate tiles with 3 chains, measured
  // slower here, 245 vs 211 us at 32 -> 32, unlike k_conv3d_fwd16).  (Persistent step
  // shares as in k_conv3d_fwd16 measured no gain at 32 -> 32, 186 vs 184 us, and the loop they need cost
  // the 64 -> 64 kernel 107 -> 144 us: not used.)
  constexpr int NTv = 256;  // only the measured best (256 threads) is instantiated
  const int NC = NTv == 512 ? 3 : 5;
  const int G = C / 16;
  S1Args a{};
  a.x = x, a.W = W, a.bias = bias, a.add = add, a.y = y, a.D = D, a.H = H, a.Wd = Wd;
  a.flip = flip;
  a.addsn = add_sn;
  a.PX = Wd + 8;
  a.MG = G == 2 ? 1 : 4;  // 32: both output tiles in the block; 64: one tile per block, 4 block groups
  size_t lds = 0;
  // rows per step: the most whose positions fit one round of the block's NWG x NC position tiles
  int YB = std::max(1, 16 * NC * (NTv / 256) / Wd);
  for (; YB >= 1; --YB) {
    a.RX = (YB + 2) * a.PX;
    while ((a.RX & 31) != 16) ++a.RX;
    lds = (size_t)4 * (3 * C * a.RX + (NTv / 64) * NC * 256 + 64);
    if (lds <= 163840) break;
  }
  if (YB < 1) return TB_ERR_UNSUPPORTED_SIZE;
  a.YB = YB > H ? H : YB;
  a.nyb = (H + a.YB - 1) / a.YB;
  a.zlen = zseg(D, N * a.nyb * a.MG, 1, 2);
  a.ZS = (D + a.zlen - 1) / a.zlen;
  const int nl = (C * (a.YB + 2) * (Wd / 4) + NTv - 1) / NTv;
  void (*kern)(S1Args) = nullptr;
#define TB_NL(k)                                                                                      \
  case k:                                                                                             \
    kern = add ? (G == 2 ? k_conv3d_mfma_s1<2, 5, k, 256, true> : k_conv3d_mfma_s1<4, 5, k, 256, true>) \
               : (G == 2 ? k_conv3d_mfma_s1<2, 5, k, 256> : k_conv3d_mfma_s1<4, 5, k, 256>);             \
    break;
  switch (nl) {
    TB_NL(1) TB_NL(2) TB_NL(3) TB_NL(4) TB_NL(5) TB_NL(6) TB_NL(7) TB_NL(8) TB_NL(9) TB_NL(10) TB_NL(11) TB_NL(12)
    default: return TB_ERR_UNSUPPORTED_SIZE;
  }
#undef TB_NL
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, dim3((unsigned)(N * a.nyb * a.MG * a.ZS)), dim3(NTv), lds,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}
