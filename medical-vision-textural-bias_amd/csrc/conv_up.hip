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

template <int CIN, int MOUT, int TY, int WV>  // WV: most float4 per input row (Wi <= 4 WV)
__global__ __launch_bounds__(256) void k_conv_s2_fewin(S2Args a) {
  static_assert(MOUT % 2 == 0, "packed output pairs");
  constexpr int NR = 2 * TY + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x;
  constexpr int PX = 4 * WV + 12, SS = CIN * NR * PX;  // row pitch (odd multiple of 4), slot stride
  float* ring = smem;                        // [5][CIN][NR][PX], input column xi at xi + 4
  for (int i = tid; i < 5 * SS; i += 256) ring[i] = 0.f;  // halos, padding rows stay 0
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
  constexpr int NL = (CIN * NR * WV + 255) / 256;
  int gof[NL], lof[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + 256 * j;
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
      const float4 v = src[gof[j] < 0 ? 0 : gof[j]];
      r[j] = (in && gof[j] >= 0) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int zi, const float4 (&r)[NL]) {
    float* d = ring + ((zi + 5) % 5) * SS;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      if (gof[j] >= 0) *reinterpret_cast<float4*>(d + lof[j]) = r[j];
  };
  __syncthreads();  // zero fill before any slab store
  load(2 * z0 - 1, ra);
  store(2 * z0 - 1, ra);
  load(2 * z0, ra);
  load(2 * z0 + 1, rb);
  // this thread's output position: row y0 + oy, column ox
  const int Wo = a.Wo, oy = tid / Wo, ox = tid - oy * Wo;
  const bool act = oy < TY && y0 + oy < a.Ho;
  const int roff = (2 * oy) * PX + 2 * ox + 3;  // + (ty PX + tx): input row 2 oy + ty, column 2 ox + tx - 1
  f2v bias2[MOUT / 2];
#pragma unroll
  for (int m = 0; m < MOUT / 2; ++m)
    bias2[m] = a.bias ? f2v{a.bias[2 * m], a.bias[2 * m + 1]} : f2v{0.f, 0.f};
  const int64_t oplane = (int64_t)a.Ho * Wo;
  float* outb = a.out + (int64_t)n * MOUT * a.Do * oplane + (int64_t)(y0 + oy) * Wo + ox;
  for (int z = z0; z < z1; ++z) {
    store(2 * z, ra);
    store(2 * z + 1, rb);
    __syncthreads();
    if (z + 1 < z1) {
      load(2 * z + 2, ra);
      load(2 * z + 3, rb);
    }
    if (act) {
      // the position's 27 CIN inputs into registers, then one packed FMA chain per output pair
      float v[CIN * 27];
#pragma unroll
      for (int tz = 0; tz < 3; ++tz) {
        const float* sl = ring + ((2 * z - 1 + tz + 5) % 5) * SS + roff;
#pragma unroll
        for (int c = 0; c < CIN; ++c)
#pragma unroll
          for (int ty = 0; ty < 3; ++ty)
#pragma unroll
            for (int tx = 0; tx < 3; ++tx) v[c * 27 + tz * 9 + ty * 3 + tx] = sl[(c * NR + ty) * PX + tx];
      }
      const cf2v_p kp = (cf2v_p)(cfloat_p)a.K;
      float* o = outb + (int64_t)z * oplane;
#pragma unroll
      for (int m = 0; m < MOUT / 2; ++m) {
        f2v acc = bias2[m];
#pragma unroll
        for (int k = 0; k < CIN * 27; ++k) acc = __builtin_elementwise_fma(f2v{v[k], v[k]}, kp[m * CIN * 27 + k], acc);
        o[(int64_t)(2 * m) * a.Do * oplane] = acc.x;
        o[(int64_t)(2 * m + 1) * a.Do * oplane] = acc.y;
      }
    }
    __syncthreads();  // every wave is done with this step's slots before the next step's stores
  }
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

template <int MO, int TY, int WV>
__global__ __launch_bounds__(256) void k_convT_fewout(TArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = (int)threadIdx.x;
  constexpr int PX = 4 * WV + 8, CS = (TY + 1) * PX;
  const int Cin = a.Cin, SS = Cin * CS;
  float* ring = smem;            // [3][Cin][TY + 1][PX], column xi at xi + 4 (xi = Wi: zero)
  for (int i = tid; i < 3 * SS; i += 256) ring[i] = 0.f;
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
  constexpr int NL = (32 * (TY + 1) * WV + 255) / 256;
  const int nitem = Cin * (TY + 1) * W4;
  int gof[NL], lof[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + 256 * j;
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
      const float4 v = src[gof[j] < 0 ? 0 : gof[j]];
      rg[j] = (in && gof[j] >= 0) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int zi) {
    float* d = ring + (zi % 3) * SS;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      if (gof[j] >= 0) *reinterpret_cast<float4*>(d + lof[j]) = rg[j];
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
      const float* s0 = ring + (z % 3) * SS + roff;
      const float* s1 = ring + ((z + 1) % 3) * SS + roff;
#pragma unroll 1
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
  auto kern = k_conv_s2_fewin<CIN, MOUT, TY, WV>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  const int per_cu = lds <= 81920 ? 2 : 1;
  a.zlen = zseg(a.Do, N * a.nyb, per_cu, 1);
  a.ZS = (a.Do + a.zlen - 1) / a.zlen;
  hipLaunchKernelGGL(kern, dim3((unsigned)(N * a.nyb * a.ZS)), dim3(256), lds, st, a);
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
  const size_t lds = (size_t)4 * 5 * Cin * a.RR * a.PX;
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
  const int TY = 256 / Wi >= 3 ? 3 : 256 / Wi >= 2 ? 2 : 1;
  TArgs a{};
  a.x = x, a.W = W, a.bias = bias, a.y = y;
  a.Cin = Cin, a.Di = Di, a.Hi = Hi, a.Wi = Wi;
  a.PX = 4 * (Wi <= 80 ? 20 : 32) + 8;  // = the kernel's compile-time pitch
  a.CS = (TY + 1) * a.PX;
  a.nyb = (Hi + TY - 1) / TY;
  const size_t lds = (size_t)4 * 3 * Cin * a.CS;
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
  if (!kern) return TB_ERR_UNSUPPORTED_SIZE;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return TB_ERR_HIP;
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, a);
  return hipGetLastError() == hipSuccess ? TB_OK : TB_ERR_HIP;
}
