// kern_wrap.hip -- separable route for wrap-only programs (wrap.h).
//
// Reference: WrapArtifact.__call__ (source_code/filters_and_operators.py:503-515): FFT, shift, every
// odd shifted index of each axis times alpha, inverse shift, inverse FFT, `.real`.  The three masks
// are symmetric 1-D masks, so y = T_h T_w T_d x with T a real circulant per axis (wrap.h):
//   k_wrap_even   D even: per (bc, quad of rows, 4 columns) the 8 voxels {h, h+H/2} x {w, w+W/2} x
//                 {d, d+D/2} in, the 8 outputs of the 2-tap products out
//   k_wrap_dgemm  D odd: per unit = one quad of 4-row chunks (16 image rows), the 2-tap H/W combine
//                 at load time, then the D circulant as split-f16 MFMA products
// Algorithmic bytes: 4 B per voxel in, 4 B per stored column (D + pad) out.
#include "wrap.h"

#include <cfloat>
#include <cmath>
#include <map>
#include <mutex>


namespace tb {

namespace {

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 h16x2v __attribute__((ext_vector_type(2)));

constexpr float WRAP_K_SCALE = 64.f;  // circulant entries x 2^6 before the f16 split (lo parts stay normal)

__device__ __forceinline__ void split_f16(float x, _Float16& h, _Float16& l) {
  h = (_Float16)x;
  l = (_Float16)(x - (float)h);
}

// Workgroup's per-sample (min, max) as order-preserving keys in LDS (ds_min / ds_max).
__device__ __forceinline__ void keys_add(uint32_t* keys, int s, float lo, float hi) {
  atomicMin(&keys[2 * s], f2key(lo));
  atomicMax(&keys[2 * s + 1], f2key(hi));
}

// The workgroup's partials out, count-in, and the last workgroup's reduction into a.mm (the keys
// of samples bc0 / C .. + nb).  Called by every thread after its last keys_add.
__device__ void wrap_keys_out(const WrapArgs& a, uint32_t* keys, int nb) {
  __shared__ int last;
  __shared__ float red[2 * WRAP_NT / 64];
  __syncthreads();  // every wave's LDS key updates done
  const int tid = (int)threadIdx.x;
  if (tid < nb) {   // lanes of wave 0
    const uint32_t kl = keys[2 * tid], kh = keys[2 * tid + 1];
    store_partial(a.mmp + (int64_t)blockIdx.x * TB_MAX_BATCH + tid,
                  make_float2(kl == 0xffffffffu ? FLT_MAX : key2f(kl), kh == 0u ? -FLT_MAX : key2f(kh)));
  }
  if (tid == 0) last = arrive_last(a.cnt, gridDim.x);  // wave 0's partial stores drained inside
  __syncthreads();
  if (!last) return;
  const int lane = tid & 63, wid = tid >> 6;
  for (int i = 0; i < nb; ++i) {
    float lo = FLT_MAX, hi = -FLT_MAX;
    for (int g = tid; g < (int)gridDim.x; g += WRAP_NT) {
      const float2 v = load_partial(a.mmp + (int64_t)g * TB_MAX_BATCH + i);
      lo = fminf(lo, v.x);
      hi = fmaxf(hi, v.y);
    }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (lane == 0) {
      red[wid] = lo;
      red[WRAP_NT / 64 + wid] = hi;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < WRAP_NT / 64; ++w) {
        lo = fminf(lo, red[w]);
        hi = fmaxf(hi, red[WRAP_NT / 64 + w]);
      }
      const int sb = a.bc0 / a.C + i;
      a.mm[2 * sb] = f2key(lo);
      a.mm[2 * sb + 1] = f2key(hi);
    }
    __syncthreads();
  }
}

}  // namespace

// ------------------------------------------------------------------------------------ D odd
// Unit u = (bc, hq < H/2, gq < ceil(W/8)): role r = (rh, rw) holds rows (hq + rh H/2, 4 gq + rw W/2 + g),
// g < nrow <= 4.  Image row n = 4 r + g of the unit is the MFMA column n = lane & 15.
//   A = K^T fragment: lane (row d_out = 16 t + (lane & 15), k = d_in = 32 s + 8 (lane >> 4) + j) =
//       k[(d_out - d_in) mod D] = Tab[m], m = d_in - d_out: 8 consecutive entries, read from the copy
//       c = -lane mod 8 of the table that makes the lane's start 16-B aligned;
//   B = X^T fragment: lane (column n, k = d_in) from the unit's staged, combined, scaled rows;
//   C: lane (column n, rows d_out = 16 t + 4 (lane >> 4) + 0..3) -- 4 consecutive columns of one
//       output row: one 16-B store.
// Per-sample 2-tap weights in LDS: w[s][0..3] = (a_h a_w, b_h a_w, a_h b_w, b_h b_w), w[s][4..5] = (a_d, b_d)
// (a dynamically indexed kernel-argument array would otherwise sit in SGPRs and spill)
__device__ __forceinline__ void wrap_weights(const WrapArgs& a, float (*w)[8]) {
  const int t = (int)threadIdx.x;
  if (t < TB_MAX_BATCH) {
    w[t][0] = a.ah[t] * a.aw[t];
    w[t][1] = a.bh[t] * a.aw[t];
    w[t][2] = a.ah[t] * a.bw[t];
    w[t][3] = a.bh[t] * a.bw[t];
    w[t][4] = a.ad[t];
    w[t][5] = a.bd[t];
  }
}

template <int NTO, int KS, bool VEC>
__global__ __launch_bounds__(WRAP_NT) __attribute__((amdgpu_waves_per_eu(NTO <= 10 ? 3 : 2, 8))) void k_wrap_dgemm(WrapArgs) {
  const WrapArgs& a = kargs<WrapArgs>();
  constexpr int L = (32 * KS + 16 * NTO + 8 + 15) & ~15;  // halfs per table copy
  constexpr int OFF = 16 * NTO + 8;                       // Tab index of m = 0 is OFF - c in copy c
  constexpr int NF = (16 * NTO + 63) / 64;                // float4 slots per lane and role chunk (4 D <= 64 NTO)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* tab = reinterpret_cast<_Float16*>(smem);     // [hi, lo][8 copies][L]
  __shared__ uint32_t keys[2 * TB_MAX_BATCH];
  __shared__ float wts[TB_MAX_BATCH][8];
  wrap_weights(a, wts);
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, W = a.W, D = a.D;
  const int nb = a.nbc / a.C;
  for (int i = tid; i < 8 * L; i += WRAP_NT) {
    const int c = i / L, idx = i - c * L;
    const int m = idx + c - OFF;
    int j = (-m) % D;
    j += j < 0 ? D : 0;
    const double v = (j == 0 ? 1.0 : 0.0) + ((double)a.alpha - 1.0) * a.q[j];
    _Float16 h, l;
    split_f16((float)(v * (double)WRAP_K_SCALE), h, l);
    tab[c * L + idx] = h;
    tab[(8 + c) * L + idx] = l;
  }
  if (tid < 2 * TB_MAX_BATCH) keys[tid] = (tid & 1) ? 0u : 0xffffffffu;
  __syncthreads();
  float* stg = reinterpret_cast<float*>(smem + 2 * 8 * L * 2) + wv * a.region;

  const int Hh = H / 2, Wh = W / 2, NG = (Wh + 3) / 4;
  const int per_bc = Hh * NG;
  const int nunit = a.nbc * per_bc;
  const int per = (nunit + (int)gridDim.x - 1) / (int)gridDim.x;
  const int ub = (int)blockIdx.x * per, ue = ub + per < nunit ? ub + per : nunit;
  const int ncolo = D + a.ypad;
  const bool vst = a.vec & 2;
  const FastDiv fd = FastDiv::make(D);

  const int n = lane & 15, role = n >> 2, g = n & 3, kb = lane >> 4;
  const int cpy = (-lane) & 7;
  const _Float16* thp = tab + cpy * L + (OFF - cpy + 8 * kb - n) - 16 * (NTO - 1);  // + 32 s + 16 (NTO - 1 - t)
  const float* xrd = stg + role * a.RS + g * D + 8 * kb;                            // + 32 s + j
  int cur = -1;
  float lo = FLT_MAX, hi = -FLT_MAX;
  // the quad's four role chunks (rows 4 gq + rw W/2 + g of slabs hq + rh H/2) of unit u into v
  auto load_unit = [&](int u, float4 (&v)[4][NF]) {
    const int bcl = u / per_bc, rem = u - bcl * per_bc, hq = rem / NG, gq = rem - hq * NG;
    const int bc = a.bc0 + bcl;
    const int nrow = Wh - 4 * gq < 4 ? Wh - 4 * gq : 4, len = nrow * D;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* xr = a.x + (int64_t)bc * a.xsbc + (int64_t)(hq + (r & 1) * Hh) * a.xsh +
                        (int64_t)(4 * gq + (r >> 1) * Wh) * a.xsw;
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int e = 4 * (lane + 64 * i);
        if (VEC && nrow == 4) {  // contiguous rows, 4 D floats (a multiple of 4): clamped 16-B loads, no branch
          const int f = lane + 64 * i;
          const float4 q4 = *reinterpret_cast<const float4*>(xr + 4 * (f < D ? f : D - 1));
          v[r][i] = f < D ? q4 : make_float4(0.f, 0.f, 0.f, 0.f);
        } else if (VEC) {  // the last, partial chunk of a row block: clamped scalar loads
          float t[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float z = xr[e + q < len ? e + q : len - 1];
            t[q] = e + q < len ? z : 0.f;
          }
          v[r][i] = make_float4(t[0], t[1], t[2], t[3]);
        } else {
          float t[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ee = e + q, gg = fd.div(ee);
            t[q] = ee < len ? xr[(int64_t)gg * a.xsw + (ee - gg * D)] : 0.f;
          }
          v[r][i] = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
    }
  };
  float4 v[4][NF];
  if (ub + wv < ue) load_unit(ub + wv, v);
  for (int u = ub + wv; u < ue; u += WRAP_NT / 64) {
    const int bcl = u / per_bc, rem = u - bcl * per_bc, hq = rem / NG, gq = rem - hq * NG;
    const int bc = a.bc0 + bcl, sl = bcl / a.C;
    const int nrow = Wh - 4 * gq < 4 ? Wh - 4 * gq : 4;
    const float w00 = wts[sl][0], w10 = wts[sl][1], w01 = wts[sl][2], w11 = wts[sl][3];
    // the H / W 2-tap combine at load time (it commutes with T_d; 4 FMAs per voxel, as packed f32 pairs)
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const f32x4v x0 = {v[0][i].x, v[0][i].y, v[0][i].z, v[0][i].w}, x1 = {v[1][i].x, v[1][i].y, v[1][i].z, v[1][i].w};
      const f32x4v x2 = {v[2][i].x, v[2][i].y, v[2][i].z, v[2][i].w}, x3 = {v[3][i].x, v[3][i].y, v[3][i].z, v[3][i].w};
      const f32x4v y0 = w00 * x0 + w10 * x1 + w01 * x2 + w11 * x3;
      const f32x4v y1 = w10 * x0 + w00 * x1 + w11 * x2 + w01 * x3;
      const f32x4v y2 = w01 * x0 + w11 * x1 + w00 * x2 + w10 * x3;
      const f32x4v y3 = w11 * x0 + w01 * x1 + w10 * x2 + w00 * x3;
#pragma unroll
      for (int c = 0; c < 4; ++c) mx = max3_abs(max3_abs(mx, y0[c], y1[c]), y2[c], y3[c]);
      v[0][i] = make_float4(y0[0], y0[1], y0[2], y0[3]);
      v[1][i] = make_float4(y1[0], y1[1], y1[2], y1[3]);
      v[2][i] = make_float4(y2[0], y2[1], y2[2], y2[3]);
      v[3][i] = make_float4(y3[0], y3[1], y3[2], y3[3]);
    }
    // per-unit power of two: max |scaled| < 2^14 (f16 hi parts in range, lo parts normal)
    int ex;
    (void)frexpf(wave_max(mx), &ex);
    const float sx = ldexpf(1.f, 14 - ex), inv = ldexpf(1.f, ex - 14) * (1.f / WRAP_K_SCALE);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int f = lane + 64 * i;
        if (f < D) {  // 4 f < 4 D: inside the role's 4-row chunk
          const f32x4v s4 = f32x4v{v[r][i].x, v[r][i].y, v[r][i].z, v[r][i].w} * sx;
          *reinterpret_cast<f32x4v*>(stg + r * a.RS + 4 * f) = s4;
        }
      }
    // the wave's next unit: its loads fly during this unit's products and stores
    if (u + WRAP_NT / 64 < ue) load_unit(u + WRAP_NT / 64, v);
    // ---- T_d: Y^T = K^T X^T in split f16.  K is Toeplitz: the A fragment of (k-step s, tile t) is the
    // table at 16 j, j = 2 s + NTO - 1 - t.  The tiles are done in two halves of NTH (20 accumulator
    // registers live, not 40 -- at 3 waves per SIMD a spill reload here waited out the next unit's
    // loads); per half each distinct fragment is read from LDS once and used for every (s, t) on its
    // diagonal against the B fragments of all KS k-steps held in registers (per tile the s order, and so
    // the sums, are those of an s-outer loop).
    const bool rowok = g < nrow;
    h16x8 bh[KS], bl[KS];
    // k-steps inside D for every row of a full unit read without predicates (wave-uniform test); the
    // rest compare against a per-unit opaque limit (loop-invariant compares would be hoisted out of the
    // unit loop as 2 SGPRs of lane mask each, spilled to VGPR lanes)
    int lim = rowok ? D - 8 * kb : 0;
    asm volatile("" : "+v"(lim));
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float xv[8];
      if (nrow == 4 && 32 * s + 32 <= D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = xrd[32 * s + j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = 32 * s + j < lim ? xrd[32 * s + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; j += 2) {  // packed conversions: v_cvt_pk_f16_f32
        const f32x2v p = {xv[j], xv[j + 1]};
        const h16x2v h = __builtin_convertvector(p, h16x2v);
        const h16x2v l = __builtin_convertvector(p - __builtin_convertvector(h, f32x2v), h16x2v);
        bh[s][j] = h[0];
        bh[s][j + 1] = h[1];
        bl[s][j] = l[0];
        bl[s][j + 1] = l[1];
      }
    }
    // ---- epilogue setup: output row n, columns 16 t + 4 kb + 0..3 (zero past D), per-sample min/max
    if (sl != cur) {  // wave-uniform
      if (cur >= 0) {
        const float l2 = wave_min(lo), h2 = wave_max(hi);
        if (lane == 0) keys_add(keys, cur, l2, h2);
      }
      cur = sl;
      lo = FLT_MAX;
      hi = -FLT_MAX;
    }
    float* yrow = a.y + (int64_t)bc * a.ysbc + (int64_t)(hq + (role & 1) * Hh) * a.ysh +
                  (int64_t)(4 * gq + (role >> 1) * Wh + g) * a.ysw;
    // Tiles whose 16 columns are all image columns, in a unit whose 16 rows all exist (wave-uniform),
    // store and reduce without per-lane predicates; the rest compare against per-lane limits that are
    // opaque to the compiler (hoisted out of the unit loop, the compares became SGPR-pair masks that
    // spilled to VGPR lanes and came back by ~240 v_readlane per unit).
    int dq = D - 4 * kb, nq = ncolo - 4 * kb;  // column 16 t + 4 kb + r is an image / stored column
    asm volatile("" : "+v"(dq), "+v"(nq));
    const int dqr = rowok ? dq : -(1 << 20), nqr = rowok ? nq : -(1 << 20);
    const bool full = nrow == 4;
    int Dv = D, nco = ncolo;  // per-unit copies: the tiles' uniform tests are not hoisted (and spilled) either
    asm volatile("" : "+s"(Dv), "+s"(nco));
    auto store_tile = [&](int t, const f32x4v& av) {
      if (16 * t >= nco) return;  // wave-uniform
      const int d0 = 16 * t + 4 * kb;
      float o[4];
      if (full && 16 * t + 16 <= Dv) {  // wave-uniform fast path
        const f32x4v ov = av * inv;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = ov[r];
        lo = min3_raw(min3_raw(lo, o[0], o[1]), o[2], o[3]);
        hi = max3_raw(max3_raw(hi, o[0], o[1]), o[2], o[3]);
        if (vst) {
          *reinterpret_cast<f32x4v*>(yrow + d0) = ov;
          return;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = 16 * t + r < dq ? av[r] * inv : 0.f;
          const bool in = 16 * t + r < dqr;
          lo = fminf(lo, in ? o[r] : FLT_MAX);
          hi = fmaxf(hi, in ? o[r] : -FLT_MAX);
        }
      }
      if (vst && 16 * t + 16 <= nco) {  // wave-uniform: the whole tile inside the stored row
        if (rowok) *reinterpret_cast<f32x4v*>(yrow + d0) = f32x4v{o[0], o[1], o[2], o[3]};
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * t + r < nqr) yrow[d0 + r] = o[r];
      }
    };
    constexpr int NTH = NTO / 2;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int t0 = NTH * hf;
      __builtin_amdgcn_sched_barrier(0);  // the halves are not interleaved by the scheduler
      f32x4v acc[NTH];
#pragma unroll
      for (int i = 0; i < NTH; ++i) acc[i] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 2 * KS + NTO - 2; ++j) {
        if (j < NTO - t0 - NTH || j > 2 * KS - 2 + NTO - 1 - t0) continue;  // no tile of this half (compile-time)
        const h16x8 kh = *reinterpret_cast<const h16x8*>(thp + 16 * j);
        const h16x8 kl = *reinterpret_cast<const h16x8*>(thp + 8 * L + 16 * j);
        // the three split products of the diagonal's pairs interleaved (consecutive MFMAs on different
        // accumulators); per accumulator the order kh bl, kl bh, kh bh is kept
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int t = NTO - 1 - (j - 2 * s);
            if (t < t0 || t >= t0 + NTH) continue;  // compile-time
            acc[t - t0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(p == 1 ? kl : kh, p == 0 ? bl[s] : bh[s],
                                                                 acc[t - t0], 0, 0, 0);
          }
      }
#pragma unroll
      for (int i = 0; i < NTH; ++i) store_tile(t0 + i, acc[i]);
    }
  }
  if (!a.mm) return;
  if (cur >= 0) {
    const float l2 = wave_min(lo), h2 = wave_max(hi);
    if (lane == 0) keys_add(keys, cur, l2, h2);
  }
  wrap_keys_out(a, keys, nb);
}

// ------------------------------------------------------------------------------------ D even
// Item = (bc, hq < H/2, wq < W/2, 4 columns j4 of d < D/2): the 8 rows-x-halves of one octet,
// 4 columns each.  y(r, e) = sum_{r', e'} wgt(r ^ r') (e == e' ? ad : bd) x(r', e').
__global__ __launch_bounds__(WRAP_NT) void k_wrap_even(WrapArgs) {
  const WrapArgs& a = kargs<WrapArgs>();
  __shared__ uint32_t keys[2 * TB_MAX_BATCH];
  __shared__ float wts[TB_MAX_BATCH][8];
  wrap_weights(a, wts);
  const int tid = (int)threadIdx.x;
  if (tid < 2 * TB_MAX_BATCH) keys[tid] = (tid & 1) ? 0u : 0xffffffffu;
  __syncthreads();
  const int H = a.H, W = a.W, D = a.D;
  const int Hh = H / 2, Wh = W / 2, Dh = D / 2, ND4 = (Dh + 3) / 4;
  const int64_t per_bc = (int64_t)Hh * Wh * ND4;
  const int64_t nitem = (int64_t)a.nbc * per_bc;
  const int64_t per = (nitem + gridDim.x - 1) / gridDim.x;
  const int64_t ib = (int64_t)blockIdx.x * per, ie = ib + per < nitem ? ib + per : nitem;
  const bool vld = (a.vec & 1) && (Dh & 3) == 0, vst = (a.vec & 2) && (Dh & 3) == 0;
  int cur = -1;
  float lo = FLT_MAX, hi = -FLT_MAX;
  for (int64_t it = ib + tid; it < ie; it += WRAP_NT) {
    const int bcl = (int)(it / per_bc);
    int rem = (int)(it - bcl * per_bc);
    const int j4 = rem % ND4;
    rem /= ND4;
    const int wq = rem % Wh, hq = rem / Wh;
    const int bc = a.bc0 + bcl, sl = bcl / a.C;
    const float w00 = wts[sl][0], w10 = wts[sl][1], w01 = wts[sl][2], w11 = wts[sl][3];
    const float ad = wts[sl][4], bd = wts[sl][5];
    const int d0 = 4 * j4;
    float xv[4][2][4];
    const float* xr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      xr[r] = a.x + (int64_t)bc * a.xsbc + (int64_t)(hq + (r & 1) * Hh) * a.xsh + (int64_t)(wq + (r >> 1) * Wh) * a.xsw;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float* p = xr[r] + d0 + e * Dh;
        if (vld) {
          const float4 q = *reinterpret_cast<const float4*>(p);
          xv[r][e][0] = q.x, xv[r][e][1] = q.y, xv[r][e][2] = q.z, xv[r][e][3] = q.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) xv[r][e][q] = d0 + q < Dh ? p[q] : 0.f;
        }
      }
    }
    if (sl != cur) {
      if (cur >= 0) keys_add(keys, cur, lo, hi);
      cur = sl;
      lo = FLT_MAX;
      hi = -FLT_MAX;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* yr = a.y + (int64_t)bc * a.ysbc + (int64_t)(hq + (r & 1) * Hh) * a.ysh + (int64_t)(wq + (r >> 1) * Wh) * a.ysw;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float s0 = 0.f, s1 = 0.f;  // same / other half
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) {
            const int x = r ^ r2;
            const float wt = x == 0 ? w00 : (x == 1 ? w10 : (x == 2 ? w01 : w11));
            s0 += wt * xv[r2][e][q];
            s1 += wt * xv[r2][e ^ 1][q];
          }
          o[q] = ad * s0 + bd * s1;
        }
        float* p = yr + d0 + e * Dh;
        if (vst) {
          *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (d0 + q < Dh) p[q] = o[q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (d0 + q < Dh) {
            lo = fminf(lo, o[q]);
            hi = fmaxf(hi, o[q]);
          }
      }
      if (j4 == 0)
        for (int p = 0; p < a.ypad; ++p) yr[D + p] = 0.f;
    }
  }
  if (!a.mm) return;
  if (cur >= 0) keys_add(keys, cur, lo, hi);
  wrap_keys_out(a, keys, a.nbc / a.C);
}

// ------------------------------------------------------------------------------------ host
bool wrap_program(const tb_sample_ops& s, float* alpha) {
  if (s.n < 1) return false;
  float al = 1.f;
  for (int o = 0; o < s.n; ++o) {
    const tb_op& op = s.op[o];
    if (op.kind != TB_OP_WRAP || op.chan >= 0) return false;
    al *= op.f[0];
  }
  if (alpha) *alpha = al;
  return true;
}

bool wrap_shape_ok(int H, int W, int D, int ypad) {
  if (H < 2 || W < 2 || (H & 1) || (W & 1) || D < 1) return false;
  return !(D & 1) || D + ypad <= WRAP_MAX_COLS;
}

void wrap_q_table(int D, double* q) {
  const double pi = 3.14159265358979323846;
  for (int j = 0; j < D; ++j) {
    double s = 0.0;
    for (int f = 0; f < D; ++f)
      if (((f + D / 2) % D) & 1) s += std::cos(2.0 * pi * (double)(((int64_t)f * j) % D) / (double)D);
    q[j] = s / (double)D;
  }
}

namespace {
template <class K>
int wrap_occupancy(K kern, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  const auto key = std::make_pair(reinterpret_cast<const void*>(kern), lds);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, WRAP_NT, lds) != hipSuccess || occ < 1) occ = 1;
  occ = occ > 8 ? 8 : occ;
  cache[key] = occ;
  return occ;
}

template <int NTO, int KS>
hipError_t launch_dgemm(WrapArgs& a, int ncu, hipStream_t st) {
  constexpr int L = (32 * KS + 16 * NTO + 8 + 15) & ~15;
  const bool vec = a.vec & 1;
  a.RS = (4 * a.D + 3) & ~3;
  a.region = (3 * a.RS + 3 * a.D + 32 * KS + 3) & ~3;
  const size_t lds = (size_t)32 * L + (size_t)4 * a.region * (WRAP_NT / 64);
  auto kern = vec ? k_wrap_dgemm<NTO, KS, true> : k_wrap_dgemm<NTO, KS, false>;
  const hipError_t e = allow_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int Wh = a.W / 2, NG = (Wh + 3) / 4;
  const int64_t nunit = (int64_t)a.nbc * (a.H / 2) * NG;
  int grid = ncu * wrap_occupancy(kern, lds);
  const int64_t need = (nunit + WRAP_NT / 64 - 1) / (WRAP_NT / 64);
  if (grid > need) grid = (int)need;
  if (grid > WRAP_MAX_WG) grid = WRAP_MAX_WG;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(WRAP_NT), lds, st, a);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_wrap(WrapArgs& a, const float* alpha, int nb, int ncu, hipStream_t st) {
  const int n[3] = {a.H, a.W, a.D};
  float* av[3] = {a.ah, a.aw, a.ad};
  float* bv[3] = {a.bh, a.bw, a.bd};
  for (int i = 0; i < nb; ++i)
    for (int ax = 0; ax < 3; ++ax) {
      const float al = alpha[i];
      const float sgn = ((n[ax] / 2) & 1) ? -1.f : 1.f;  // (-1)^(n/2): the roll's sign
      av[ax][i] = 0.5f * (1.f + al);
      bv[ax][i] = sgn * 0.5f * (1.f - al);
    }
  a.alpha = alpha[0];
  if (a.mm) {
    const hipError_t e = hipMemsetAsync(a.cnt, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
  }
  if (!(a.D & 1)) {
    const int64_t nitem = (int64_t)a.nbc * (a.H / 2) * (a.W / 2) * ((a.D / 2 + 3) / 4);
    int64_t grid = (int64_t)ncu * 8;
    const int64_t need = (nitem + WRAP_NT - 1) / WRAP_NT;
    grid = grid > need ? need : grid;
    grid = grid > WRAP_MAX_WG ? WRAP_MAX_WG : (grid < 1 ? 1 : grid);
    hipLaunchKernelGGL(k_wrap_even, dim3((unsigned)grid), dim3(WRAP_NT), 0, st, a);
    return hipGetLastError();
  }
  if (a.D + a.ypad <= 160) return launch_dgemm<10, 5>(a, ncu, st);
  return launch_dgemm<16, 8>(a, ncu, st);
}

}  // namespace tb
