// conv_gemm.hip -- the U-Net's channel-deep convolutions as implicit GEMMs on the f32 matrix cores.
//
// The reference's MONAI UNet (10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199; module tree
// source_code/test.ipynb:754-1010) has, besides the full-resolution layers of conv_up.hip, the
// stride-2 entries of levels 1-3 (16 -> 32, 32 -> 64, 64 -> 128, each twice: the unit and its
// residual), the bottom unit (128 -> 256, 256 -> 256, a 1x1x1 128 -> 256 residual) and the
// ConvTranspose3d ups (384 -> 64, 128 -> 32).  MIOpen/CK ran them at 23-51 TFLOP/s plus NCDHW <->
// NDHWC transposes (~4.5 ms of a 17.2 ms C3 step, forward and input gradient included).  Here every
// one of them, and every input gradient, is one kernel:
//
//   Y[m][q] = bias[m] + add[m][q] + sum_{k < K} A[m][k] X~[k][q]          (q: GEMM position, k = (c, tap))
//
// with X~ gathered from the NCDHW input on the fly (no im2col buffer): position q = (n, oz, oy, ox) of
// the position grid, tap j of the class's tap list with offsets (dz, dy, dx), input voxel
// (S oz + dz, S oy + dy, S ox + dx) (zero outside), output voxel (ymul oz + pz, ymul oy + py, ymul ox + px):
//   * Conv3d 3x3x3 / 1x1x1, stride S, padding 1 / 0: one class, taps (tz - 1, ty - 1, tx - 1), A = W;
//   * the input gradient of a stride-1 Conv3d: A[c][m t] = W[m][c][26 - t] (packed by k_cg_pack);
//   * ConvTranspose3d(stride 2, padding 1, output_padding 1) forward -- and, with a stride-2 Conv3d's
//     weight, that layer's input gradient -- in sub-pixel form: 8 parity classes (pz, py, px), per axis
//     parity 0 takes tap 1 at offset 0, parity 1 taps 2 (offset 0) and 0 (offset +1); position grid =
//     the input grid, ymul = 2, A_cls[m][c T_cls + j] = W[c][m][tap_j]: every multiply-add a real tap.
//
// k runs tap-major (k = tap Cin + c, A packed to match by k_cg_pack; Cin % 8 == 0), so the 8 k rows a
// wave gathers per stage are 8 channels of ONE tap: the tap's offset and every lane's validity bit are
// per stage, the 8 loads per lane one base address plus channel strides.  Tiling: a 256-thread block
// computes a BM x BP tile of Y over k stages of 32: A rows staged by float4 loads, X~ gathered by scalar
// loads (each lane's positions fixed for the block), both stored to LDS as [row][k parity][16 steps]
// so that each lane reads its 16 operands of a stage as four 16-B reads.  The waves (WGM x 4/WGM) own TM x TN tiles
// of 32 x 32 on mfma_f32_32x32x2f32 (exact f32: one rounding per product, as a k-ordered fmaf chain).
// Stages are double-buffered (the next stage's global loads in registers while the current one runs
// from LDS; one barrier per stage).  Small GEMMs split k over nsplit slices into float partials summed
// by k_cg_reduce (which adds bias / add and scatters to the output grid).  Blocks are numbered so that
// the m tiles of one position tile land on one XCD (its L2 serves the X~ re-reads).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "texbias.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 32;    // k rows per stage
constexpr int NTH = 256;  // threads per block
constexpr int RS = 36;    // LDS floats per tile row: 32 k + 4 pad (16-B reads of 16 rows hit distinct banks)

struct CGArgs {
  const float* x;
  const float* A;
  const float* bias;
  const float* add;
  float* y;
  float* part;
  int64_t xsn, ysn, addsn;  // batch strides (floats); channel strides below
  int64_t xbytes;           // bytes of x from its base (the gather's buffer range)
  int xsc, ysc;
  int Cin, M;
  int IDm, IH, IW;  // input extents
  int OD, OH, OW;   // position grid
  int YH, YW;       // output H, W extents
  int S, ymul;
  int P;            // N OD OH OW
  int nsplit, kper, mtiles, ptiles, ncls;
  int kind;  // taps: 0 = 3x3x3 (tz - 1, ty - 1, tx - 1), 1 = 1x1x1, 2 = sub-pixel class (parity bits = class)
  int64_t aoff[8];
  int Kc[8], Tc[8];
};

// tap j of class cls: input offsets and the weight's tap index (host and device)
__host__ __device__ inline void tap_of(int kind, int cls, int j, int& dz, int& dy, int& dx, int& widx) {
  if (kind == 0) {
    dz = j / 9 - 1, dy = (j / 3) % 3 - 1, dx = j % 3 - 1, widx = j;
  } else if (kind == 1) {
    dz = dy = dx = 0, widx = 0;
  } else {
    // parity 0: tap 1 at offset 0; parity 1: i = 0 -> tap 2 at offset 0, i = 1 -> tap 0 at offset +1
    const int pz = (cls >> 2) & 1, py = (cls >> 1) & 1, px = cls & 1;
    const int nx = 1 + px, ny = 1 + py;
    const int ix = j % nx, iy = (j / nx) % ny, iz = j / (nx * ny);
    dz = pz ? iz : 0, dy = py ? iy : 0, dx = px ? ix : 0;
    const int tz = pz ? (iz ? 0 : 2) : 1, ty = py ? (iy ? 0 : 2) : 1, tx = px ? (ix ? 0 : 2) : 1;
    widx = tz * 9 + ty * 3 + tx;
  }
}

__device__ __forceinline__ int xcd_remap(int b, int nb) {
  // hardware dispatch sends block b to XCD b % 8: give XCD x the contiguous logical range of blocks
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

template <int BM, int BP, int WGM>
__global__ __launch_bounds__(NTH) void k_conv_gemm(const CGArgs a) {
  constexpr int WGN = 4 / WGM;
  constexpr int TM = BM / WGM / 32, TN = BP / WGN / 32;
  constexpr int NPOS = BP / 64;          // gather positions per lane
  constexpr int AQ = BM * KC / 4 / NTH;  // A float4 per thread per stage
  static_assert(TM >= 1 && TN >= 1 && NPOS >= 1 && AQ >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  constexpr int LBUF = (BM + BP) * RS;   // floats per stage buffer
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int b = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int mt = b % a.mtiles;
  b /= a.mtiles;
  const int pt = b % a.ptiles;
  b /= a.ptiles;
  const int split = b % a.nsplit, cls = b / a.nsplit;
  const int T = a.Tc[cls], K = a.Kc[cls], Kld = K;
  const float* __restrict__ A = a.A + a.aoff[cls];
  const int Cin = a.Cin;
  const int k_beg = split * a.kper;
  const int k_end = min(K, k_beg + a.kper);
  const int m0 = mt * BM, p0 = pt * BP;
  const int IHW = a.IH * a.IW;

  // gather positions: lane + 64 i of the tile; byte offset of the tap-(0,0,0) voxel of channel 0 and the
  // per-tap validity bits
  int xo[NPOS];
  uint32_t vm[NPOS];
#pragma unroll
  for (int i = 0; i < NPOS; ++i) {
    const int p = p0 + lane + 64 * i;
    const bool ok = p < a.P;
    int t = ok ? p : 0;
    const int ox = t % a.OW;
    t /= a.OW;
    const int oy = t % a.OH;
    t /= a.OH;
    const int oz = t % a.OD, n = t / a.OD;
    const int bz = a.S * oz, by = a.S * oy, bx = a.S * ox;
    xo[i] = 4 * ((int)(n * a.xsn) + bz * IHW + by * a.IW + bx);
    uint32_t m = 0;
    for (int j = 0; j < T; ++j) {
      int dz, dy, dx, wi;
      tap_of(a.kind, cls, j, dz, dy, dx, wi);
      const int iz = bz + dz, iy = by + dy, ix = bx + dx;
      const bool v = ok && iz >= 0 && iz < a.IDm && iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW;
      m |= (v ? 1u : 0u) << j;
    }
    vm[i] = m;
  }
  // the input through a buffer descriptor: an out-of-range offset reads 0 (the zero padding and the
  // k rows past k_end), so the gather needs no selects
  const uint32_t xbytes = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.xbytes);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, (int)xbytes, 0x00020000);
  const int xsc4 = 4 * a.xsc;

  // two register slots: the loads of stage s + 2 are in flight while stage s runs from LDS and stage
  // s + 1 (loaded one stage earlier) is written to the other LDS buffer.  LDS rows hold k in natural
  // order; the MFMA step st pairs k = st (lanes 0-31) with k = 16 + st (lanes 32-63).
  float rb[2][NPOS][8];
  f32x4 ra[2][AQ];
  auto gather = [&](auto SL, int k0) {
    constexpr int sl = decltype(SL)::value;
    // rows k0 + 8 w .. + 7: channels c .. c + 7 of tap t (Cin % 8 == 0)
    const int k = k0 + 8 * w;
    const int t = k / Cin, c = k - t * Cin;
    const bool kin = k < k_end;
    int dz, dy, dx, wi;
    tap_of(a.kind, cls, kin ? t : 0, dz, dy, dx, wi);
    const int off = 4 * ((dz * a.IH + dy) * a.IW + dx);
    const int soff = c * xsc4;
#pragma unroll
    for (int i = 0; i < NPOS; ++i) {
      const bool v = kin && ((vm[i] >> t) & 1u);
      const int vo = v ? xo[i] + off : (int)0x80000000;
#pragma unroll
      for (int r = 0; r < 8; ++r)
        rb[sl][i][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, soff + r * xsc4, 0));
    }
  };
  const uint32_t abytes = (uint32_t)__builtin_amdgcn_readfirstlane((int)(4 * (int64_t)a.M * Kld));
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, (int)abytes, 0x00020000);
  auto aload = [&](auto SL, int k0) {
    constexpr int sl = decltype(SL)::value;
#pragma unroll
    for (int u = 0; u < AQ; ++u) {
      const int q4 = tid + NTH * u, row = q4 % BM, kq = k0 + 4 * (q4 / BM);
      const int m = m0 + row;
      const int vo = (m < a.M && kq < k_end) ? 4 * (m * Kld + kq) : (int)0x80000000;
      ra[sl][u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, vo, 0, 0));
    }
  };
  auto stage_store = [&](auto SL) {  // slot sl -> LDS buffer sl (stage s uses slot and buffer s & 1)
    constexpr int sl = decltype(SL)::value;
    float* L = lds_dyn + sl * LBUF;
#pragma unroll
    for (int u = 0; u < AQ; ++u) {
      const int q4 = tid + NTH * u, row = q4 % BM, c4 = q4 / BM;
      *reinterpret_cast<f32x4*>(L + row * RS + 4 * c4) = ra[sl][u];
    }
#pragma unroll
    for (int i = 0; i < NPOS; ++i) {
      float* d = L + (BM + lane + 64 * i) * RS + 8 * w;
      *reinterpret_cast<f32x4*>(d) = f32x4{rb[sl][i][0], rb[sl][i][1], rb[sl][i][2], rb[sl][i][3]};
      *reinterpret_cast<f32x4*>(d + 4) = f32x4{rb[sl][i][4], rb[sl][i][5], rb[sl][i][6], rb[sl][i][7]};
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

  const int wm = w % WGM, wn = w / WGM;
  const int kk = lane >> 5, l32 = lane & 31;
  // steps h*8 .. h*8+7 of the stage in LDS buffer sl
  auto compute_half = [&](auto SL, auto H) {
    constexpr int sl = decltype(SL)::value, h = decltype(H)::value;
    const float* L = lds_dyn + sl * LBUF;
    f32x4 af[TM][2], bf[TN][2];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const float* src = L + ((wm * TM + tm) * 32 + l32) * RS + 16 * kk + 8 * h;
#pragma unroll
      for (int q = 0; q < 2; ++q) af[tm][q] = *reinterpret_cast<const f32x4*>(src + 4 * q);
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const float* src = L + (BM + (wn * TN + tn) * 32 + l32) * RS + 16 * kk + 8 * h;
#pragma unroll
      for (int q = 0; q < 2; ++q) bf[tn][q] = *reinterpret_cast<const f32x4*>(src + 4 * q);
    }
#pragma unroll
    for (int st = 0; st < 8; ++st)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm][st >> 2][st & 3], bf[tn][st >> 2][st & 3],
                                                             acc[tm][tn], 0, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  const int nst = k_beg < k_end ? (k_end - k_beg + KC - 1) / KC : 0;
  if (nst > 0) {
    gather(I0{}, k_beg);
    aload(I0{}, k_beg);
    stage_store(I0{});
    gather(I1{}, k_beg + KC);
    aload(I1{}, k_beg + KC);
  }
  __syncthreads();
  // stage s: its first 8 MFMA steps, then the loads of stage s + 2 (past the end they read zeros through
  // the descriptors' range check: no branches), the last 8 steps, stage s + 1 to the other LDS buffer
  auto body = [&](auto SL, int s) {
    using O = std::integral_constant<int, 1 - decltype(SL)::value>;
    compute_half(SL, I0{});
    gather(SL, k_beg + (s + 2) * KC);
    aload(SL, k_beg + (s + 2) * KC);
    compute_half(SL, I1{});
    stage_store(O{});
    __syncthreads();
  };
  for (int s = 0; s < nst; s += 2) {
    body(I0{}, s);
    if (s + 1 < nst) body(I1{}, s + 1);
  }

  // epilogue: C column = position (lane & 31), rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int p = p0 + (wn * TN + tn) * 32 + l32;
    if (p >= a.P) continue;
    if (a.nsplit > 1) {
      float* dst = a.part + ((int64_t)(cls * a.nsplit + split) * a.M) * a.P + p;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * TM + tm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * kk;
          if (m < a.M) dst[(int64_t)m * a.P] = acc[tm][tn][r];
        }
      continue;
    }
    int t = p;
    const int ox = t % a.OW;
    t /= a.OW;
    const int oy = t % a.OH;
    t /= a.OH;
    const int oz = t % a.OD, n = t / a.OD;
    const int pc = a.kind == 2 ? cls : 0;
    const int64_t sp = ((int64_t)(a.ymul * oz + (pc >> 2)) * a.YH + (a.ymul * oy + ((pc >> 1) & 1))) * a.YW +
                       a.ymul * ox + (pc & 1);
    float* yo = a.y + n * a.ysn + sp;
    const float* ad = a.add ? a.add + n * a.addsn + sp : nullptr;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + tm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * kk;
        if (m < a.M) {
          float v = acc[tm][tn][r] + (a.bias ? a.bias[m] : 0.f);
          if (ad) v += ad[(int64_t)m * a.ysc];
          yo[(int64_t)m * a.ysc] = v;
        }
      }
  }
}

// y = bias + add + sum of the split partials, scattered to the output grid; one thread per (cls, m, q)
__global__ __launch_bounds__(256) void k_cg_reduce(const CGArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)a.M * a.P;
  if (i >= per * a.ncls) return;
  const int cls = (int)(i / per);
  const int64_t r = i - cls * per;
  const int m = (int)(r / a.P), p = (int)(r - (int64_t)m * a.P);
  const float* src = a.part + (int64_t)cls * a.nsplit * per + (int64_t)m * a.P + p;
  float v = a.bias ? a.bias[m] : 0.f;
  float s = 0.f;
  for (int k = 0; k < a.nsplit; ++k) s += src[k * per];
  v += s;
  int t = p;
  const int ox = t % a.OW;
  t /= a.OW;
  const int oy = t % a.OH;
  t /= a.OH;
  const int oz = t % a.OD, n = t / a.OD;
  const int pc = a.kind == 2 ? cls : 0;
  const int64_t sp =
      ((int64_t)(a.ymul * oz + (pc >> 2)) * a.YH + (a.ymul * oy + ((pc >> 1) & 1))) * a.YW + a.ymul * ox + (pc & 1);
  if (a.add) v += a.add[n * a.addsn + (int64_t)m * a.ysc + sp];
  a.y[n * a.ysn + (int64_t)m * a.ysc + sp] = v;
}

// Packed A operands, k tap-major: A_cls[m][j Cin + c] = W(m, c, tap_j of cls).  mode 0 (Conv3d, W
// [M][Cin][T]): W[m][c][widx]; mode 1 (input gradient of a stride-1 conv whose weight is Wl [Cin][M][T]):
// Wl[c][m][T - 1 - widx]; mode 2 (sub-pixel classes, Wt [Cin][M][27]): Wt[c][m][widx].
__global__ __launch_bounds__(256) void k_cg_pack(const float* __restrict__ W, float* __restrict__ out, int mode,
                                                 int64_t total, const CGArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  int cls = 0;
  while (cls + 1 < a.ncls && i >= a.aoff[cls + 1]) ++cls;
  const int64_t r = i - a.aoff[cls];
  const int Kc = a.Kc[cls], T = a.Tc[cls], Cin = a.Cin, M = a.M;
  const int m = (int)(r / Kc), k = (int)(r - (int64_t)m * Kc);
  const int j = k / Cin, c = k - j * Cin;
  int dz, dy, dx, wi;
  tap_of(a.kind, cls, j, dz, dy, dx, wi);
  const int TW = a.kind == 1 ? 1 : 27;  // taps in the weight tensor
  (void)T;
  float v;
  if (mode == 0) v = W[((int64_t)m * Cin + c) * TW + wi];
  else if (mode == 1) v = W[((int64_t)c * M + m) * TW + (TW - 1 - wi)];
  else v = W[((int64_t)c * M + m) * 27 + wi];
  out[i] = v;
}

int g_ncu = 0;
int num_cu() {
  static std::once_flag once;
  std::call_once(once, [] {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&g_ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
      g_ncu = 256;
  });
  return g_ncu > 0 ? g_ncu : 256;
}

struct Plan {
  CGArgs a;
  int BM, BP, WGM;
  size_t pack_floats, part_floats;
};

inline size_t align_floats(size_t n) { return (n + 63) & ~size_t(63); }
inline size_t lds_bytes(int BM, int BP) { return (size_t)2 * (BM + BP) * RS * sizeof(float); }

// Fill the geometry and tiling of a call (no device pointers).  Returns TB_OK or an error code.
int make_plan(int mode, int N, int Cin, int M, int D, int H, int Wd, int stride, int ksize, Plan& pl) {
  if (N < 1 || Cin < 1 || M < 1 || D < 1 || H < 1 || Wd < 1) return TB_ERR_INVALID_ARG;
  if (mode < 0 || mode > 2 || (ksize != 3 && ksize != 1) || (stride != 1 && stride != 2)) return TB_ERR_INVALID_ARG;
  if (Cin % 8 != 0) return TB_ERR_UNSUPPORTED_SIZE;
  if (mode == 2 && (ksize != 3 || stride != 2)) return TB_ERR_INVALID_ARG;
  if (mode == 1 && stride != 1) return TB_ERR_INVALID_ARG;
  CGArgs& a = pl.a;
  a = CGArgs{};
  a.Cin = Cin, a.M = M, a.IDm = D, a.IH = H, a.IW = Wd;
  a.xsc = D * H * Wd;
  if ((int64_t)N * Cin * D * H * Wd >= (int64_t)1 << 31) return TB_ERR_UNSUPPORTED_SIZE;
  if (mode == 2) {
    a.S = 1, a.ymul = 2, a.OD = D, a.OH = H, a.OW = Wd, a.YH = 2 * H, a.YW = 2 * Wd, a.ncls = 8, a.kind = 2;
    int64_t off = 0;
    for (int cls = 0; cls < 8; ++cls) {
      const int T = (1 + ((cls >> 2) & 1)) * (1 + ((cls >> 1) & 1)) * (1 + (cls & 1));
      a.Tc[cls] = T, a.Kc[cls] = Cin * T, a.aoff[cls] = off;
      off += (int64_t)M * Cin * T;
    }
    pl.pack_floats = (size_t)off;
  } else {
    const int pad = ksize == 3 ? 1 : 0;
    a.S = stride, a.ymul = 1, a.ncls = 1, a.kind = ksize == 3 ? 0 : 1;
    a.OD = (D + 2 * pad - ksize) / stride + 1, a.OH = (H + 2 * pad - ksize) / stride + 1,
    a.OW = (Wd + 2 * pad - ksize) / stride + 1;
    a.YH = a.OH, a.YW = a.OW;
    const int T = ksize * ksize * ksize;
    a.Tc[0] = T, a.Kc[0] = Cin * T, a.aoff[0] = 0;
    pl.pack_floats = (size_t)M * Cin * T;
  }
  a.ysc = a.ymul == 2 ? 8 * a.OD * a.OH * a.OW : a.OD * a.OH * a.OW;
  if ((int64_t)N * M * a.ysc >= (int64_t)1 << 31) return TB_ERR_UNSUPPORTED_SIZE;
  a.P = N * a.OD * a.OH * a.OW;
  // tile: M <= 32 -> 32 x 128; M <= 64 -> 64 x 64; else 128 x 128
  const int tile = M <= 32 ? 1 : (M <= 64 ? 2 : 5);
  static const int cfg[6][3] = {{0, 0, 0}, {32, 128, 1}, {64, 64, 2}, {128, 64, 2}, {64, 128, 2}, {128, 128, 2}};
  pl.BM = cfg[tile][0], pl.BP = cfg[tile][1], pl.WGM = cfg[tile][2];
  a.mtiles = (M + pl.BM - 1) / pl.BM;
  a.ptiles = (a.P + pl.BP - 1) / pl.BP;
  int Kmax = 0;
  for (int c = 0; c < a.ncls; ++c) Kmax = a.Kc[c] > Kmax ? a.Kc[c] : Kmax;
  // split k to minimise (rounds of the chip's block slots) x (stages per block + a fixed per-block cost
  // of ~3 stages: position decode, tap masks, partial stores); ties keep the smaller split
  const int64_t base = (int64_t)a.mtiles * a.ptiles * a.ncls;
  int occ = (int)(163840 / lds_bytes(pl.BM, pl.BP));
  occ = occ > 4 ? 4 : (occ < 1 ? 1 : occ);
  const int64_t slots = (int64_t)occ * num_cu();
  const int stages = (Kmax + KC - 1) / KC;
  double best = 1e30;
  int ns = 1;
  for (int s = 1; s <= 16 && s <= stages; ++s) {
    const int64_t blocks = base * s;
    const int64_t rounds = (blocks + slots - 1) / slots;
    const double cost = (double)rounds * ((stages + s - 1) / s + 3);
    if (cost < best * 0.97) best = cost, ns = s;
  }
  a.kper = ((Kmax + ns - 1) / ns + KC - 1) / KC * KC;
  a.nsplit = (Kmax + a.kper - 1) / a.kper;
  pl.part_floats = a.nsplit > 1 ? (size_t)a.ncls * a.nsplit * M * a.P : 0;
  return TB_OK;
}

template <int BM, int BP, int WGM>
hipError_t launch_tile(const CGArgs& a, hipStream_t st) {
  const int64_t nb = (int64_t)a.mtiles * a.ptiles * a.nsplit * a.ncls;
  const size_t lds = lds_bytes(BM, BP);
  static std::once_flag once;
  static hipError_t attr = hipSuccess;
  std::call_once(once, [&] {
    attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv_gemm<BM, BP, WGM>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  });
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_conv_gemm<BM, BP, WGM>), dim3((unsigned)nb), dim3(NTH), lds, st, a);
  return hipGetLastError();
}

}  // namespace

size_t tb_conv3d_gemm_workspace_bytes(int mode, int N, int Cin, int M, int D, int H, int Wd, int stride, int ksize) {
  Plan pl;
  if (make_plan(mode, N, Cin, M, D, H, Wd, stride, ksize, pl) != TB_OK) return 0;
  return 4 * (align_floats(pl.pack_floats) + align_floats(pl.part_floats)) + 256;
}

int tb_conv3d_gemm_f32(int mode, const float* x, int64_t xsn, const float* W, const float* bias, const float* add,
                       int64_t addsn, float* y, int64_t ysn, int N, int Cin, int M, int D, int H, int Wd, int stride,
                       int ksize, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !W || !y) return TB_ERR_INVALID_ARG;
  Plan pl;
  const int rc = make_plan(mode, N, Cin, M, D, H, Wd, stride, ksize, pl);
  if (rc != TB_OK) return rc;
  CGArgs& a = pl.a;
  const size_t need = 4 * (align_floats(pl.pack_floats) + align_floats(pl.part_floats)) + 256;
  if (!ws || ws_bytes < need) return TB_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  a.x = x, a.bias = bias, a.add = add, a.y = y;
  a.xsn = xsn > 0 ? xsn : (int64_t)Cin * a.xsc;
  a.ysn = ysn > 0 ? ysn : (int64_t)M * a.ysc;
  a.addsn = addsn > 0 ? addsn : a.ysn;
  a.xbytes = 4 * ((int64_t)(N - 1) * a.xsn + (int64_t)Cin * a.xsc);
  if (a.xbytes >= (int64_t)1 << 31) return TB_ERR_UNSUPPORTED_SIZE;
  float* wsf = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  {
    const int64_t total = (int64_t)pl.pack_floats;
    hipLaunchKernelGGL(k_cg_pack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, wsf, mode, total, a);
    a.A = wsf;
  }
  a.part = wsf + align_floats(pl.pack_floats);
  hipError_t e = hipSuccess;
  if (pl.BM == 32) e = launch_tile<32, 128, 1>(a, st);
  else if (pl.BM == 64 && pl.BP == 64) e = launch_tile<64, 64, 2>(a, st);
  else if (pl.BM == 64) e = launch_tile<64, 128, 2>(a, st);
  else if (pl.BP == 64) e = launch_tile<128, 64, 2>(a, st);
  else e = launch_tile<128, 128, 2>(a, st);
  if (e != hipSuccess) return TB_ERR_HIP;
  if (a.nsplit > 1) {
    const int64_t tot = (int64_t)a.ncls * a.M * a.P;
    hipLaunchKernelGGL(k_cg_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, a);
    if (hipGetLastError() != hipSuccess) return TB_ERR_HIP;
  }
  return TB_OK;
}

int tb_conv3d_gemm_config(int mode, int N, int Cin, int M, int D, int H, int Wd, int stride, int ksize, int64_t* cfg) {
  Plan pl;
  const int rc = make_plan(mode, N, Cin, M, D, H, Wd, stride, ksize, pl);
  if (rc != TB_OK || !cfg) return rc != TB_OK ? rc : TB_ERR_INVALID_ARG;
  cfg[0] = pl.BM, cfg[1] = pl.BP, cfg[2] = pl.a.nsplit, cfg[3] = pl.a.kper;
  cfg[4] = (int64_t)pl.a.mtiles * pl.a.ptiles * pl.a.nsplit * pl.a.ncls;
  cfg[5] = pl.a.P;
  return TB_OK;
}
