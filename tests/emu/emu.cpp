// Host emulator of the texbias kernels -- TEST INFRASTRUCTURE ONLY.
//
// Compiles medical-vision-textural-bias_amd/csrc/{fft_core,slab_ct,plan_host,sap_core}.h with the host
// clang++ and runs the same per-workgroup bodies the gfx950 kernels run, one workgroup at a time with
// a single "thread" and a no-op barrier (the compile-time slab passes: their item functions, phase by
// phase, in the device kernels' order).  Each phase of a body consists of independent work items (in-place
// butterflies own their slots), so the result equals the device schedule's.  This lets the CPU
// suite check indexing, packing, op programs and the RNG against the oracle without a GPU.
// Never loaded by the product package.
#include <cmath>
#include <algorithm>
#include <cstring>
#include <vector>

#include "fft_core.h"
#include "plan_host.h"
#include "sap_core.h"
#include "slab_ct.h"
#include "kspace_ct.h"

using namespace tb;

namespace {
struct HostCtx {
  int tid = 0, nthreads = 1;
  void sync() {}
};

int make_plan(int H, int W, int D, PlanTables& pt, tb_plan_dev& pl) {
  int rc = build_tables(H, W, D, pt);
  if (rc) return rc;
  pl.H = H; pl.W = W; pl.D = D; pl.pad = 0;
  for (int a = 0; a < 3; ++a) { pl.ax[a] = pt.ax[a]; pl.tw[a] = pt.tw[a].data(); }
  pl.rev_d = pt.rev_d.data();
  pl.irev_h = pt.irev_h.data();
  pl.irev_w = pt.irev_w.data();
  return TB_OK;
}

using ct::v2;

// pass A / C of one (bc, h) slab through the compile-time plan's item functions
template <int W, int D>
void ct_slab_fwd(const tb_plan_dev& pl, v2* lds, const float* xb, int64_t sw, v2* Sb) {
  using P = ct::SlabPlan<W, D>;
  HostCtx ctx;
  ct::load_tw<P>(ctx, lds, pl);
  v2 r[P::R0];
  for (int it = 0; it < P::N_F0; ++it) { ct::a_load<P>(r, xb, sw, it); ct::a_f0<P>(lds, r, it); }
  if constexpr (P::FUSED_DU) {
    std::vector<v2> rd(2 * (size_t)P::R1 * P::N_DU);
    for (int it = 0; it < P::N_DU; ++it) ct::a_du_load<P>(lds, &rd[2 * P::R1 * it], it);
    for (int it = 0; it < P::N_DU; ++it) ct::a_du_compute<P>(lds, &rd[2 * P::R1 * it], it);
  } else {
    for (int it = 0; it < P::N_D1; ++it) ct::a_d1<P>(lds, it);
    std::vector<v2> ru(2 * (size_t)P::N_U);
    for (int it = 0; it < P::N_U; ++it) ct::a_u_read<P>(lds, &ru[2 * it], it);
    for (int it = 0; it < P::N_U; ++it) ct::a_u_write<P>(lds, &ru[2 * it], it);
  }
  for (int it = 0; it < P::N_W0; ++it) ct::a_w0<P>(lds, it);
  for (int it = 0; it < P::N_W1; ++it) ct::a_w1<P>(lds, Sb, it);
}

template <int W, int D>
void ct_slab_inv(const tb_plan_dev& pl, v2* lds, const v2* Sb, float* yb, int64_t sw, int ypad, float scale,
                 float& lo, float& hi) {
  using P = ct::SlabPlan<W, D>;
  HostCtx ctx;
  ct::load_tw<P>(ctx, lds, pl);
  v2 r[P::Q1];
  for (int it = 0; it < P::N_W1; ++it) { ct::c_load<P>(r, Sb, it); ct::c_g0<P>(lds, r, it); }
  for (int it = 0; it < P::N_W0; ++it) ct::c_g1<P>(lds, it);
  if constexpr (P::FUSED_DU) {
    std::vector<v2> rd(2 * (size_t)P::R1 * P::N_DU);
    for (int it = 0; it < P::N_DU; ++it) ct::c_re_load<P>(lds, &rd[2 * P::R1 * it], it);
    for (int it = 0; it < P::N_DU; ++it) ct::c_re_compute<P>(lds, &rd[2 * P::R1 * it], it);
  } else {
    std::vector<v2> ru(2 * (size_t)P::N_U);
    for (int it = 0; it < P::N_U; ++it) ct::c_r_read<P>(lds, &ru[2 * it], it);
    for (int it = 0; it < P::N_U; ++it) ct::c_r_write<P>(lds, &ru[2 * it], it);
    for (int it = 0; it < P::N_D1; ++it) ct::c_e1<P>(lds, it);
  }
  for (int it = 0; it < P::N_F0; ++it) ct::c_e0<P>(lds, yb, sw, scale, it, lo, hi);
  for (int w = 0; w < W; ++w)
    for (int d = D; d < D + ypad; ++d) yb[w * sw + d] = 0.f;
}

// pass B of one (bc, tile of T columns) through the compile-time tile plan's item functions
template <int H>
void ct_tile(const tb_plan_dev& pl, v2* lds, v2* S, int bc, int tile, const tb_sample_ops& so, int chan) {
  constexpr int T = ct::kCtTileT;
  using P = ct::TilePlan<H, T>;
  const int ncols = pl.W * (pl.D / 2 + 1);
  const int j0 = tile * T, nc = (ncols - j0) < T ? (ncols - j0) : T;
  v2* Sc = S + (int64_t)bc * H * ncols + j0;
  for (int i = 0; i < H; ++i) lds[P::OFF_TW + i] = ct::V(pl.tw[0][i].x, pl.tw[0][i].y);
  for (int it = 0; it < P::N0; ++it) {
    v2 r[P::Q0];
    for (int q = 0; q < P::Q0; ++q) r[q] = ct::V(0.f, 0.f);
    if (it % T < nc) ct::b_load<P>(r, Sc, ncols, it);
    ct::b_s0<P>(lds, r, it);
  }
  const int mk = ct::mask_kind(&so, 1);  // the device's unrolled middle phase for mask-only programs
  for (int it = 0; it < P::NM; ++it) {
    const int c = it % T;
    const FreqCol fc = ct::tile_col(pl, j0 + (c < nc ? c : 0));
    if (mk == ct::MASK_GIBBS) ct::b_mid_mask<P, ct::MASK_GIBBS>(lds, so, chan, fc, it);
    else if (mk == ct::MASK_LAYER) ct::b_mid_mask<P, ct::MASK_LAYER>(lds, so, chan, fc, it);
    else if (mk == ct::MASK_DISK) ct::b_mid_mask<P, ct::MASK_DISK>(lds, so, chan, fc, it);
    else ct::b_mid<P>(lds, so, chan, fc, it);
  }
  for (int it = 0; it < P::N0; ++it)
    if (it % T < nc) ct::b_s1<P>(lds, Sc, ncols, it);
}
#define TB_EMU_CT_TILE_H(X) TB_CT_TILE_H(X) X(20) X(36)
bool ct_tile_has(int H) {
#define TB_X(h) if (H == h) return true;
  TB_EMU_CT_TILE_H(TB_X)
#undef TB_X
  return false;
}
size_t ct_tile_lds_cf(int H) {
#define TB_X(h) if (H == h) return ct::TilePlan<h, ct::kCtTileT>::TOTAL;
  TB_EMU_CT_TILE_H(TB_X)
#undef TB_X
  return 0;
}
void ct_tile_run(int H, const tb_plan_dev& pl, v2* lds, v2* S, int bc, int tile, const tb_sample_ops& so, int chan) {
#define TB_X(h) if (H == h) return ct_tile<h>(pl, lds, S, bc, tile, so, chan);
  TB_EMU_CT_TILE_H(TB_X)
#undef TB_X
}

// the device library's shapes plus small test shapes (odd/even D, composite and prime radices)
#define TB_EMU_CT_SHAPES(X) TB_CT_SLAB_SHAPES(X) X(240, 155) X(24, 35) X(20, 28)  // (240, 155): host-only since round 6

bool ct_has(int W, int D) {
#define TB_X(w, d) if (W == w && D == d) return true;
  TB_EMU_CT_SHAPES(TB_X)
#undef TB_X
  return false;
}
size_t ct_lds_cf(int W, int D) {
#define TB_X(w, d) if (W == w && D == d) return ct::SlabPlan<w, d>::TOTAL;
  TB_EMU_CT_SHAPES(TB_X)
#undef TB_X
  return 0;
}
void ct_fwd(int W, int D, const tb_plan_dev& pl, v2* lds, const float* xb, int64_t sw, v2* Sb) {
#define TB_X(w, d) if (W == w && D == d) return ct_slab_fwd<w, d>(pl, lds, xb, sw, Sb);
  TB_EMU_CT_SHAPES(TB_X)
#undef TB_X
}
void ct_inv(int W, int D, const tb_plan_dev& pl, v2* lds, const v2* Sb, float* yb, int64_t sw, int ypad, float scale,
            float& lo, float& hi) {
#define TB_X(w, d) if (W == w && D == d) return ct_slab_inv<w, d>(pl, lds, Sb, yb, sw, ypad, scale, lo, hi);
  TB_EMU_CT_SHAPES(TB_X)
#undef TB_X
}
// ---- half units + split spectrum (slab_ct.h HalfPlan, kspace_ct.h b_mid_split), device phase order
template <int W, int D>
void half_fwd(const tb_plan_dev& pl, v2* lds, const float* xb, int64_t sw, v2* Sslab, int e) {
  using HP = ct::HalfPlan<W, D>;
  using P = typename HP::P;
  HostCtx ctx;
  ct::load_tw_half<HP>(ctx, lds, pl);
  float* raw = reinterpret_cast<float*>(lds);
  for (int L = 0; L < HP::NRAW; ++L) raw[L] = xb[(2 * (L / D) + e) * sw + L % D];
  std::vector<v2> rf((size_t)P::N_F0 * P::R0);
  for (int it = 0; it < P::N_F0; ++it) ct::a_load_raw<P>(raw, &rf[(size_t)P::R0 * it], it);
  for (int it = 0; it < P::N_F0; ++it) ct::a_f0<P>(lds, &rf[(size_t)P::R0 * it], it);
  if constexpr (P::FUSED_DU) {
    std::vector<v2> rd(2 * (size_t)P::R1 * P::N_DU);
    for (int it = 0; it < P::N_DU; ++it) ct::a_du_load<P>(lds, &rd[2 * P::R1 * it], it);
    for (int it = 0; it < P::N_DU; ++it) ct::a_du_compute<P>(lds, &rd[2 * P::R1 * it], it);
  } else {
    for (int it = 0; it < P::N_D1; ++it) ct::a_d1<P>(lds, it);
    std::vector<v2> ru(2 * (size_t)P::N_U);
    for (int it = 0; it < P::N_U; ++it) ct::a_u_read<P>(lds, &ru[2 * it], it);
    for (int it = 0; it < P::N_U; ++it) ct::a_u_write<P>(lds, &ru[2 * it], it);
  }
  for (int it = 0; it < P::N_W0; ++it) ct::a_w0<P>(lds, it);
  for (int it = 0; it < P::N_W1; ++it) ct::a_w1_half<HP>(lds, Sslab + (int64_t)e * HP::W2 * P::Dh, e, it);
}

template <int W, int D>
void half_inv(const tb_plan_dev& pl, v2* lds, const v2* Sslab, float* yb, int64_t sw, int ypad, float scale, int e,
              float& lo, float& hi) {
  using HP = ct::HalfPlan<W, D>;
  using P = typename HP::P;
  HostCtx ctx;
  ct::load_tw_half<HP>(ctx, lds, pl);
  v2 r[P::Q1];
  const v2* Sb = Sslab + (int64_t)e * HP::W2 * P::Dh;
  for (int it = 0; it < P::N_W1; ++it) {
    ct::c_load_half<HP>(r, Sb, it);
    ct::c_twiddle_half<HP>(lds, r, e, it);
    ct::c_g0<P>(lds, r, it);
  }
  for (int it = 0; it < P::N_W0; ++it) ct::c_g1<P>(lds, it);
  if constexpr (P::FUSED_DU) {
    std::vector<v2> rd(2 * (size_t)P::R1 * P::N_DU);
    for (int it = 0; it < P::N_DU; ++it) ct::c_re_load<P>(lds, &rd[2 * P::R1 * it], it);
    for (int it = 0; it < P::N_DU; ++it) ct::c_re_compute<P>(lds, &rd[2 * P::R1 * it], it);
  } else {
    std::vector<v2> ru(2 * (size_t)P::N_U);
    for (int it = 0; it < P::N_U; ++it) ct::c_r_read<P>(lds, &ru[2 * it], it);
    for (int it = 0; it < P::N_U; ++it) ct::c_r_write<P>(lds, &ru[2 * it], it);
    for (int it = 0; it < P::N_D1; ++it) ct::c_e1<P>(lds, it);
  }
  float* y0 = yb + (int64_t)e * sw;
  for (int it = 0; it < P::N_F0; ++it) ct::c_e0<P>(lds, y0, 2 * sw, scale, it, lo, hi);
  for (int w = 0; w < HP::W2; ++w)
    for (int d = D; d < D + ypad; ++d) y0[2 * w * sw + d] = 0.f;
}

template <int H, int W, int D>
void half_tile(const tb_plan_dev& pl, v2* lds, v2* S, int bc, int tile, const tb_sample_ops& so, int chan) {
  using HP = ct::HalfPlan<W, D>;
  using P = ct::TilePlan<H, 32>;
  constexpr int TH = 16, ncols = W * HP::Dh, nh = HP::W2 * HP::Dh;
  v2* Sc = S + (int64_t)bc * H * ncols + tile * TH;
  for (int i = 0; i < H; ++i) lds[P::OFF_TW + i] = ct::V(pl.tw[0][i].x, pl.tw[0][i].y);
  std::vector<ct::f4> r((size_t)(P::N0 / 2) * P::Q0);
  for (int it = 0; it < P::N0 / 2; ++it) ct::b_load_split<P>(&r[(size_t)P::Q0 * it], Sc, ncols, nh, it);
  for (int it = 0; it < P::N0 / 2; ++it) ct::b_s0_pair_regs<P>(lds, &r[(size_t)P::Q0 * it], it);
  const int mk = ct::mask_kind(&so, 1);
  for (int it = 0; it < P::Q0 * TH; ++it) {
    FreqCol f0, f1;
    ct::tile_col_half<HP>(tile * TH + it % TH, f0, f1);
    if (mk == ct::MASK_GIBBS) ct::b_mid_split<P, ct::MASK_GIBBS>(lds, so, chan, f0, f1, it);
    else if (mk == ct::MASK_LAYER) ct::b_mid_split<P, ct::MASK_LAYER>(lds, so, chan, f0, f1, it);
    else if (mk == ct::MASK_DISK) ct::b_mid_split<P, ct::MASK_DISK>(lds, so, chan, f0, f1, it);
    else ct::b_mid_split<P, ct::MASK_GENERIC>(lds, so, chan, f0, f1, it);
  }
  for (int it = 0; it < P::N0 / 2; ++it) ct::b_s1_split<P>(lds, Sc, ncols, nh, it);
}

// the device's half shapes (H = 240) plus a small one
#define TB_EMU_HALF_SHAPES(X) X(240, 240, 155) X(20, 48, 35)
bool half_has(int H, int W, int D) {
#define TB_X(h, w, d) if (H == h && W == w && D == d) return true;
  TB_EMU_HALF_SHAPES(TB_X)
#undef TB_X
  return false;
}
size_t half_lds_cf(int H, int W, int D) {
#define TB_X(h, w, d) if (H == h && W == w && D == d) return std::max((size_t)ct::HalfPlan<w, d>::TOTAL, (size_t)ct::TilePlan<h, 32>::TOTAL);
  TB_EMU_HALF_SHAPES(TB_X)
#undef TB_X
  return 0;
}
void half_run_fwd(int H, int W, int D, const tb_plan_dev& pl, v2* lds, const float* xb, int64_t sw, v2* Ss, int e) {
#define TB_X(h, w, d) if (H == h && W == w && D == d) return half_fwd<w, d>(pl, lds, xb, sw, Ss, e);
  TB_EMU_HALF_SHAPES(TB_X)
#undef TB_X
}
void half_run_inv(int H, int W, int D, const tb_plan_dev& pl, v2* lds, const v2* Ss, float* yb, int64_t sw, int ypad,
                  float scale, int e, float& lo, float& hi) {
#define TB_X(h, w, d) if (H == h && W == w && D == d) return half_inv<w, d>(pl, lds, Ss, yb, sw, ypad, scale, e, lo, hi);
  TB_EMU_HALF_SHAPES(TB_X)
#undef TB_X
}
void half_run_tile(int H, int W, int D, const tb_plan_dev& pl, v2* lds, v2* S, int bc, int tile, const tb_sample_ops& so,
                   int chan) {
#define TB_X(h, w, d) if (H == h && W == w && D == d) return half_tile<h, w, d>(pl, lds, S, bc, tile, so, chan);
  TB_EMU_HALF_SHAPES(TB_X)
#undef TB_X
}
}  // namespace

extern "C" {

int tbemu_radices(int n, int* out) {
  tb_axis ax;
  if (!factorize(n, ax)) return -1;
  for (int s = 0; s < ax.nst; ++s) out[s] = ax.radix[s];
  return ax.nst;
}

// same contract as tb_kspace_filter_f32, host pointers; minmax_out = float[B][2] (min, max) or NULL;
// use_ct: run passes A and C through the compile-time slab plan when (W, D) has one, pass B
// through the compile-time tile plan when H has one
int tbemu_kspace_filter_f32(int H, int W, int D, const float* x, const int64_t* xs, float* y, const int64_t* ys,
                            int y_pad, int B, int C, const tb_sample_ops* ops, float* minmax_out, int T, int use_ct) {
  PlanTables pt;
  tb_plan_dev pl;
  int rc = make_plan(H, W, D, pt, pl);
  if (rc) return rc;
  const int Dh = D / 2 + 1;
  const SlabGeo sg = slab_geo(W, D);
  if (T <= 0) T = 64;
  const TileGeo tg = tile_geo(H, T);
  const bool half = use_ct == 2 && half_has(H, W, D);
  const bool ct_on = use_ct && ct_has(W, D);
  const bool ct_b = use_ct && ct_tile_has(H);
  std::vector<cf> lds((size_t)std::max({(size_t)sg.total_cf, (size_t)tg.total_cf, ct_lds_cf(W, D), ct_tile_lds_cf(H),
                                        half_lds_cf(H, W, D)}) +
                      16);
  v2* ldsv = reinterpret_cast<v2*>(lds.data());
  std::vector<cf> S((size_t)B * C * H * W * Dh);
  HostCtx ctx;
  const float scale = (float)(1.0 / ((double)H * W * D));
  const int ntiles = (W * Dh + T - 1) / T;
  for (int b = 0; b < B; ++b) {
    float lo = 3.402823466e38f, hi = -3.402823466e38f;
    for (int c = 0; c < C; ++c) {
      const int bc = b * C + c;
      for (int h = 0; h < H && half; ++h)
        for (int e = 0; e < 2; ++e)
          half_run_fwd(H, W, D, pl, ldsv, x + bc * xs[0] + h * xs[1], xs[2],
                       reinterpret_cast<v2*>(S.data()) + ((int64_t)bc * H + h) * W * Dh, e);
      if (half) {
        for (int t = 0; t < (W / 2) * Dh / 16; ++t)
          half_run_tile(H, W, D, pl, ldsv, reinterpret_cast<v2*>(S.data()), bc, t, ops[b], c);
        for (int h = 0; h < H; ++h)
          for (int e = 0; e < 2; ++e) {
            float l = 3.402823466e38f, u = -3.402823466e38f;
            half_run_inv(H, W, D, pl, ldsv, reinterpret_cast<const v2*>(S.data()) + ((int64_t)bc * H + h) * W * Dh,
                         y + bc * ys[0] + h * ys[1], ys[2], y_pad, scale, e, l, u);
            lo = l < lo ? l : lo;
            hi = u > hi ? u : hi;
          }
        continue;
      }
      for (int h = 0; h < H; ++h) {
        if (ct_on)
          ct_fwd(W, D, pl, ldsv, x + bc * xs[0] + h * xs[1], xs[2],
                 reinterpret_cast<v2*>(S.data()) + ((int64_t)bc * H + h) * W * Dh);
        else
          pass_a_body<HostCtx, 1>(ctx, lds.data(), pl, x, xs[0], xs[1], xs[2], S.data(), bc, h);
      }
      if (ct_b) {
        const int nt = (W * Dh + ct::kCtTileT - 1) / ct::kCtTileT;
        for (int t = 0; t < nt; ++t) ct_tile_run(H, pl, ldsv, reinterpret_cast<v2*>(S.data()), bc, t, ops[b], c);
      } else {
        for (int t = 0; t < ntiles; ++t) pass_b_body<HostCtx, 1>(ctx, lds.data(), pl, S.data(), bc, t, T, ops[b], c);
      }
      for (int h = 0; h < H; ++h) {
        float l = 3.402823466e38f, u = -3.402823466e38f;
        if (ct_on)
          ct_inv(W, D, pl, ldsv, reinterpret_cast<const v2*>(S.data()) + ((int64_t)bc * H + h) * W * Dh,
                 y + bc * ys[0] + h * ys[1], ys[2], y_pad, scale, l, u);
        else
          pass_c_body<HostCtx, 1>(ctx, lds.data(), pl, S.data(), y, ys[0], ys[1], ys[2], y_pad, bc, h, scale, &l,
                                  &u);
        lo = l < lo ? l : lo;
        hi = u > hi ? u : hi;
      }
    }
    if (minmax_out) { minmax_out[2 * b] = lo; minmax_out[2 * b + 1] = hi; }
  }
  return TB_OK;
}

// Philox u01 stream for voxel counters [ctr0, ctr0 + n)
void tbemu_philox_u01(uint64_t lin0, int64_t n, uint64_t offset, uint64_t seed, float* out) {
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t L = lin0 + (uint64_t)i;
    out[i] = u01(philox(L >> 2, offset, seed).v[L & 3]);
  }
}

int tbemu_sap_class(const float* u, int64_t n, float lo, float hi, int8_t* cls) {
  for (int64_t i = 0; i < n; ++i) cls[i] = (int8_t)sap_class(u[i], lo, hi);
  return 0;
}

uint32_t tbemu_f2key(float f) { return f2key(f); }
float tbemu_key2f(uint32_t k) { return key2f(k); }
}
