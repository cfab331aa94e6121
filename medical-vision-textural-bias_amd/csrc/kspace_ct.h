// kspace_ct.h -- compile-time-planned pass B (H-axis pencils + the k-space op program).
//
// Pass B of the generic path (fft_core.h pass_b_body) with H fixed at compile time (two DIF
// stages, H = Q0*Q1, e.g. 240 = 16*15), one work item per thread per phase:
//   S0  (c, j):   H stage 0 (radix Q0, L = H/Q0) from HBM into the LDS tile [H][T]
//   MID (c, blk): last DIF stage (radix Q1) -> op program on its Q1 coefficients -> first inverse
//                 stage, all in registers; the op program runs ops-outermost over the butterfly's
//                 coefficients (one decode of each op per butterfly, geometry per coefficient)
//   S1  (c, j):   inverse H stage 0 (radix Q0) from the tile back to HBM (in place)
// Semantics of the op program are those of apply_ops (fft_core.h), which cites the reference.
#pragma once

#include "slab_ct.h"

namespace tb {
namespace ct {

template <int H_, int T_> struct TilePlan {
  static constexpr int H = H_, T = T_;
  static constexpr int Q0 = first_radix(H), Q1 = H / Q0, L = Q1;
  static_assert(two_stage(H), "H must factor as two supported radices");
  static constexpr int N0 = T * L;   // (c, j)    first DIF / last DIT stage items
  static constexpr int NM = T * Q0;  // (c, blk)  fused middle items
  static constexpr int OFF_TW = H * T;
  static constexpr int TOTAL = OFF_TW + H;
  static constexpr size_t LDS_BYTES = (size_t)TOTAL * 8;
};

// op program over the R coefficients of one butterfly; coefficient q has H frequency kh0 + kst*q
template <int R, int H, class SO>
TB_HD void ops_bfly(const SO& so, int chan, v2* v, const FreqCol& fc, int kh0, int kst) {
  v2 gb[R];
  bool in_group = false;
  for (int o = 0; o < so.n; ++o) {
    const tb_op& op = so.op[o];
    const bool spike = op.kind == TB_OP_SPIKE;
    if (spike && (!in_group || op.reserved != 1)) {
      TB_UNROLL
      for (int q = 0; q < R; ++q) gb[q] = v[q];
    }
    in_group = spike;
    if (op.chan >= 0 && op.chan != chan) continue;
    switch (op.kind) {
      case TB_OP_DISK: {
        const bool ir = op.i[0] != 0, off = op.i[1] != 0;
        TB_UNROLL
        for (int q = 0; q < R; ++q) {
          const AxisGeo h = axis_geo(kh0 + kst * q, H);
          const int sq = h.dsq + fc.dsq;
          bool in = ir ? ((int64_t)sq < op.l) : ((float)sq < op.f[0]);
          if (off) in = !in;
          v[q] = in ? v[q] : V(0.f, 0.f);
        }
      } break;
      case TB_OP_GIBBS: {
        TB_UNROLL
        for (int q = 0; q < R; ++q) {
          const AxisGeo h = axis_geo(kh0 + kst * q, H);
          const float m = 0.5f * (((int64_t)(h.ef + fc.ef) <= op.l ? 1.f : 0.f) +
                                  ((int64_t)(h.en + fc.en) <= op.l ? 1.f : 0.f));
          v[q] = m * v[q];
        }
      } break;
      case TB_OP_LAYER: {
        TB_UNROLL
        for (int q = 0; q < R; ++q) {
          const AxisGeo h = axis_geo(kh0 + kst * q, H);
          const float m = 0.5f * ((layer_in(op, h.ef + fc.ef) ? 1.f : 0.f) + (layer_in(op, h.en + fc.en) ? 1.f : 0.f));
          v[q] = m * v[q];
        }
      } break;
      case TB_OP_WRAP: {
        const float a = op.f[0];
        TB_UNROLL
        for (int q = 0; q < R; ++q) {
          const int nodd = axis_geo(kh0 + kst * q, H).odd + fc.odd;
          const float m = nodd == 0 ? 1.f : (nodd == 1 ? a : (nodd == 2 ? a * a : a * a * a));
          v[q] = m * v[q];
        }
      } break;
      case TB_OP_SPIKE: {
        if (fc.kw == op.i[1] && fc.kd == op.i[2]) {  // this column holds f (at most one coefficient)
          TB_UNROLL
          for (int q = 0; q < R; ++q) {
            if (kh0 + kst * q == op.i[0]) {
              const cf g = mk(gb[q].x, gb[q].y);
              const cf d = sub(spike_target(op, g), g);
              v[q] += 0.5f * V(d.x, d.y);
            }
          }
        }
        if (fc.nkw == op.i[1] && fc.nkd == op.i[2]) {  // ... or -f
          TB_UNROLL
          for (int q = 0; q < R; ++q) {
            if (negk(kh0 + kst * q, H) == op.i[0]) {
              const cf kf = mk(gb[q].x, -gb[q].y);
              const cf d = sub(spike_target(op, kf), kf);
              v[q] += 0.5f * V(d.x, -d.y);
            }
          }
        }
      } break;
      case TB_OP_ZF: {
        const uint64_t Wz = (uint64_t)op.i[1], Dz = (uint64_t)op.i[2], ch = (uint64_t)chan * (uint64_t)H;
        TB_UNROLL
        for (int q = 0; q < R; ++q) {
          const int kh = kh0 + kst * q;
          const float m = 0.5f * (zf_keep(op, ((ch + (uint64_t)kh) * Wz + (uint64_t)fc.kw) * Dz + (uint64_t)fc.kd) +
                                  zf_keep(op, ((ch + (uint64_t)negk(kh, H)) * Wz + (uint64_t)fc.nkw) * Dz +
                                              (uint64_t)fc.nkd));
          v[q] = m * v[q];
        }
      } break;
      default: break;
    }
  }
}

// S0 item (c, j): loads (global, column c of the tile) then DFT + twiddles into the LDS tile
template <class P>
TB_HD void b_load(v2* r, const v2* __restrict__ Sc, int64_t ncols, int it) {
  const int j = it / P::T, c = it - j * P::T;
  const v2* s = Sc + (int64_t)j * ncols + c;
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) r[q] = s[(int64_t)(q * P::L) * ncols];
}
template <class P>
TB_HD void b_s0(v2* lds, v2* a, int it) {
  const int j = it / P::T, c = it - j * P::T;
  const v2* tw = lds + P::OFF_TW;
  Dv<P::Q0, true>::run(a);
  v2* t = lds + j * P::T + c;
  t[0] = a[0];
  TB_UNROLL
  for (int q = 1; q < P::Q0; ++q) t[q * P::L * P::T] = j ? cmul(a[q], tw[j * q]) : a[q];
}
template <class P, class SO>
TB_HD void b_mid(v2* lds, const SO& so, int chan, const FreqCol& fc, int it) {
  const int blk = it / P::T, c = it - blk * P::T;
  v2* t = lds + (blk * P::L) * P::T + c;
  v2 a[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = t[q * P::T];
  Dv<P::Q1, true>::run(a);
  ops_bfly<P::Q1, P::H>(so, chan, a, fc, blk, P::Q0);  // slot blk*L + q holds kh = blk + Q0*q
  Dv<P::Q1, false>::run(a);
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) t[q * P::T] = a[q];
}
// b_mid with the op program applied one coefficient at a time from the LDS tile (a rolled loop over
// the butterfly's Q1 coefficients, apply_ops per coefficient): the fully unrolled ops_bfly keeps every
// op kind's code for all Q1 coefficients live and pins pass B at 256 VGPRs (1 wave per SIMD).
template <class P, class SO>
TB_HD void b_mid_lds(v2* lds, const SO& so, int chan, const FreqCol& fc, int it) {
  const int blk = it / P::T, c = it - blk * P::T;
  v2* t = lds + (blk * P::L) * P::T + c;
  v2 a[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = t[q * P::T];
  Dv<P::Q1, true>::run(a);
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) t[q * P::T] = a[q];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int q = 0; q < P::Q1; ++q) {  // slot blk*L + q holds kh = blk + Q0*q
    const v2 v = t[q * P::T];
    const cf o = apply_ops(so, chan, mk(v.x, v.y), fc, blk + P::Q0 * q, P::H);
    t[q * P::T] = V(o.x, o.y);
  }
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = t[q * P::T];
  Dv<P::Q1, false>::run(a);
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) t[q * P::T] = a[q];
}

// Programs made of one mask-op kind (every op GIBBS, or every op LAYER, or every op DISK): the
// ops scale or zero the butterfly's Q1 coefficients in registers between the two DFTs, fully
// unrolled (b_mid_lds's rolled per-coefficient apply_ops made pass B latency-bound: 34 K of a
// 44 K-cycle unit).  Each op is applied in program order exactly as apply_ops does (scale by
// 0 / 0.5 / 1, or select), so the results are the generic path's bit for bit.
enum { MASK_GENERIC = 0, MASK_GIBBS = 1, MASK_LAYER = 2, MASK_DISK = 3 };
template <class SO>
TB_HD int mask_kind(const SO* s, int n) {
  int k = -1;
  for (int i = 0; i < n; ++i) {
    if (s[i].n < 1) return MASK_GENERIC;
    for (int o = 0; o < s[i].n; ++o) {
      const int kd = s[i].op[o].kind;
      const int m = kd == TB_OP_GIBBS ? MASK_GIBBS : kd == TB_OP_LAYER ? MASK_LAYER : kd == TB_OP_DISK ? MASK_DISK : 0;
      if (m == 0 || (k >= 0 && m != k)) return MASK_GENERIC;
      k = m;
    }
  }
  return k < 0 ? MASK_GENERIC : k;
}
template <class P, int K, class SO>
TB_HD void b_mid_mask(v2* lds, const SO& so, int chan, const FreqCol& fc, int it) {
  const int blk = it / P::T, c = it - blk * P::T;
  v2* t = lds + (blk * P::L) * P::T + c;
  v2 a[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = t[q * P::T];
  Dv<P::Q1, true>::run(a);
  int g0[P::Q1], g1[P::Q1];  // per coefficient: (ef, en) for GIBBS / LAYER, dsq for DISK
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) {  // slot blk*L + q holds kh = blk + Q0*q
    const AxisGeo h = axis_geo(blk + P::Q0 * q, P::H);
    g0[q] = K == MASK_DISK ? h.dsq + fc.dsq : h.ef + fc.ef;
    g1[q] = h.en + fc.en;
  }
  for (int o = 0; o < so.n; ++o) {
    const tb_op& op = so.op[o];
    if (op.chan >= 0 && op.chan != chan) continue;
    if constexpr (K == MASK_GIBBS) {
      TB_UNROLL
      for (int q = 0; q < P::Q1; ++q) {
        const float m = 0.5f * (((int64_t)g0[q] <= op.l ? 1.f : 0.f) + ((int64_t)g1[q] <= op.l ? 1.f : 0.f));
        a[q] = m * a[q];
      }
    } else if constexpr (K == MASK_LAYER) {
      TB_UNROLL
      for (int q = 0; q < P::Q1; ++q) {
        const float m = 0.5f * ((layer_in(op, g0[q]) ? 1.f : 0.f) + (layer_in(op, g1[q]) ? 1.f : 0.f));
        a[q] = m * a[q];
      }
    } else {
      const bool ir = op.i[0] != 0, off = op.i[1] != 0;
      TB_UNROLL
      for (int q = 0; q < P::Q1; ++q) {
        bool in = ir ? ((int64_t)g0[q] < op.l) : ((float)g0[q] < op.f[0]);
        if (off) in = !in;
        a[q] = in ? a[q] : V(0.f, 0.f);
      }
    }
  }
  Dv<P::Q1, false>::run(a);
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) t[q * P::T] = a[q];
}

template <class P>
TB_HD void b_s1(const v2* lds, v2* __restrict__ Sc, int64_t ncols, int it) {
  const int j = it / P::T, c = it - j * P::T;
  const v2* tw = lds + P::OFF_TW;
  const v2* t = lds + j * P::T + c;
  v2 a[P::Q0];
  a[0] = t[0];
  TB_UNROLL
  for (int q = 1; q < P::Q0; ++q) a[q] = j ? cmulc(t[q * P::L * P::T], tw[j * q]) : t[q * P::L * P::T];
  Dv<P::Q0, false>::run(a);
  v2* s = Sc + (int64_t)j * ncols + c;
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) s[(int64_t)(q * P::L) * ncols] = a[q];
}

// Paired items (16-B lanes, ncols even): item it covers tile columns c = 2*cp and c+1 of row j,
// so every HBM access is one f4 (MI355X_MICROARCH.md: 8-B accesses run at 0.54-0.70x the
// 16-B rate) and a wave covers 64*16/T/8 rows of T*8 contiguous bytes.
typedef float f4 __attribute__((ext_vector_type(4)));

template <class P>
TB_HD void b_s0_pair(v2* lds, const v2* __restrict__ Sc, int64_t ncols, int it) {
  const int j = it / (P::T / 2), c = 2 * (it - j * (P::T / 2));
  const f4* s = reinterpret_cast<const f4*>(Sc + (int64_t)j * ncols + c);
  const int64_t st = (int64_t)P::L * (ncols / 2);
  v2 a[P::Q0], b[P::Q0];
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) {
    const f4 u = s[q * st];
    a[q] = V(u.x, u.y);
    b[q] = V(u.z, u.w);
  }
  const v2* tw = lds + P::OFF_TW;
  Dv<P::Q0, true>::run(a);
  Dv<P::Q0, true>::run(b);
  f4* t = reinterpret_cast<f4*>(lds + j * P::T + c);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) {
    v2 x = a[q], y = b[q];
    if (q && j) {
      const v2 w = tw[j * q];
      x = cmul(x, w);
      y = cmul(y, w);
    }
    t[q * P::L * P::T / 2] = f4{x.x, x.y, y.x, y.y};
  }
}
// b_s0_pair split in two for the persistent pass B: the loads (issued one unit ahead) and the DFT
template <class P>
TB_HD void b_load_pair(f4* r, const v2* __restrict__ Sc, int64_t ncols, int it) {
  const int j = it / (P::T / 2), c = 2 * (it - j * (P::T / 2));
  const f4* s = reinterpret_cast<const f4*>(Sc + (int64_t)j * ncols + c);
  const int64_t st = (int64_t)P::L * (ncols / 2);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) r[q] = ld_stream<TB_NT_SPEC>(s + q * st);
}
template <class P>
TB_HD void b_s0_pair_regs(v2* lds, const f4* r, int it) {
  const int j = it / (P::T / 2), c = 2 * (it - j * (P::T / 2));
  v2 a[P::Q0], b[P::Q0];
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) {
    a[q] = V(r[q].x, r[q].y);
    b[q] = V(r[q].z, r[q].w);
  }
  const v2* tw = lds + P::OFF_TW;
  Dv<P::Q0, true>::run(a);
  Dv<P::Q0, true>::run(b);
  f4* t = reinterpret_cast<f4*>(lds + j * P::T + c);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) {
    v2 x = a[q], y = b[q];
    if (q && j) {
      const v2 w = tw[j * q];
      x = cmul(x, w);
      y = cmul(y, w);
    }
    t[q * P::L * P::T / 2] = f4{x.x, x.y, y.x, y.y};
  }
}
template <class P>
TB_HD void b_s1_pair(const v2* lds, v2* __restrict__ Sc, int64_t ncols, int it) {
  const int j = it / (P::T / 2), c = 2 * (it - j * (P::T / 2));
  const v2* tw = lds + P::OFF_TW;
  const f4* t = reinterpret_cast<const f4*>(lds + j * P::T + c);
  v2 a[P::Q0], b[P::Q0];
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) {
    const f4 u = t[q * P::L * P::T / 2];
    a[q] = V(u.x, u.y);
    b[q] = V(u.z, u.w);
    if (q && j) {
      const v2 w = tw[j * q];
      a[q] = cmulc(a[q], w);
      b[q] = cmulc(b[q], w);
    }
  }
  Dv<P::Q0, false>::run(a);
  Dv<P::Q0, false>::run(b);
  f4* s = reinterpret_cast<f4*>(Sc + (int64_t)j * ncols + c);
  const int64_t st = (int64_t)P::L * (ncols / 2);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) s[q * st] = f4{a[q].x, a[q].y, b[q].x, b[q].y};
}

// column geometry of tile column c (spectrum column j0 + c = w' * Dh + kd)
TB_HD FreqCol tile_col(const tb_plan_dev& pl, int col) {
  const int Dh = pl.D / 2 + 1;
  const int wp = col / Dh;
  return freq_col(pl.irev_w[wp], col - wp * Dh, pl.W, pl.D);
}

// ------------------------------------------------------------------ split spectra (slab_ct.h HalfPlan)
// Pass B over a split spectrum: a unit is TH = T/2 first-half columns (rows w' < W/2 of the slab's
// half spectrum: E0(k'')) and their partners W/2 rows later (T1(k'')), tile columns c and c + TH.
// The middle item (blk, c < TH) forms X(k'') = E0 + T1 and X(k'' + W/2) = E0 - T1 (the last W
// butterfly, which commutes with the H stages), runs both through the last H stage, the op program
// and the first inverse H stage, and stores X'(k'') + X'(k'' + W/2), X'(k'') - X'(k'' + W/2): the
// inputs of pass C's two half units (no 1/2 -- their W/2-point inverses complete the W-point one).
template <class HP>
TB_HD void tile_col_half(int col, FreqCol& f0, FreqCol& f1) {
  const int wp = col / HP::Dh, kd = col - wp * HP::Dh;
  const int k = HP::freq(wp);
  f0 = freq_col(k, kd, HP::W, HP::D);
  f1 = freq_col(k + HP::W2, kd, HP::W, HP::D);
}

// mask-only programs (kind K) on the Q1 coefficients of butterfly blk, in registers (b_mid_mask)
template <class P, int K, class SO>
TB_HD void mask_bfly(const SO& so, int chan, const FreqCol& fc, int blk, v2* a) {
  int g0[P::Q1], g1[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) {  // slot blk*L + q holds kh = blk + Q0*q
    const AxisGeo h = axis_geo(blk + P::Q0 * q, P::H);
    g0[q] = K == MASK_DISK ? h.dsq + fc.dsq : h.ef + fc.ef;
    g1[q] = h.en + fc.en;
  }
  for (int o = 0; o < so.n; ++o) {
    const tb_op& op = so.op[o];
    if (op.chan >= 0 && op.chan != chan) continue;
    if constexpr (K == MASK_GIBBS) {
      TB_UNROLL
      for (int q = 0; q < P::Q1; ++q) {
        const float m = 0.5f * (((int64_t)g0[q] <= op.l ? 1.f : 0.f) + ((int64_t)g1[q] <= op.l ? 1.f : 0.f));
        a[q] = m * a[q];
      }
    } else if constexpr (K == MASK_LAYER) {
      TB_UNROLL
      for (int q = 0; q < P::Q1; ++q) {
        const float m = 0.5f * ((layer_in(op, g0[q]) ? 1.f : 0.f) + (layer_in(op, g1[q]) ? 1.f : 0.f));
        a[q] = m * a[q];
      }
    } else {
      const bool ir = op.i[0] != 0, off = op.i[1] != 0;
      TB_UNROLL
      for (int q = 0; q < P::Q1; ++q) {
        bool in = ir ? ((int64_t)g0[q] < op.l) : ((float)g0[q] < op.f[0]);
        if (off) in = !in;
        a[q] = in ? a[q] : V(0.f, 0.f);
      }
    }
  }
}

// middle item of a split tile; K = MASK_GENERIC applies the op program per coefficient from LDS
template <class P, int K, class SO>
TB_HD void b_mid_split(v2* lds, const SO& so, int chan, const FreqCol& f0, const FreqCol& f1, int it) {
  constexpr int TH = P::T / 2;
  const int blk = it / TH, c = it - blk * TH;
  v2* t0 = lds + (blk * P::L) * P::T + c;
  v2* t1 = t0 + TH;
  v2 a[P::Q1], b[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) {
    const v2 u = t0[q * P::T], v = t1[q * P::T];
    a[q] = u + v;
    b[q] = u - v;
  }
  Dv<P::Q1, true>::run(a);
  Dv<P::Q1, true>::run(b);
  if constexpr (K != MASK_GENERIC) {
    mask_bfly<P, K>(so, chan, f0, blk, a);
    mask_bfly<P, K>(so, chan, f1, blk, b);
  } else {
    TB_UNROLL
    for (int q = 0; q < P::Q1; ++q) {
      t0[q * P::T] = a[q];
      t1[q * P::T] = b[q];
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
    for (int q = 0; q < P::Q1; ++q) {
      const int kh = blk + P::Q0 * q;
      const v2 u = t0[q * P::T], v = t1[q * P::T];
      const cf ou = apply_ops(so, chan, mk(u.x, u.y), f0, kh, P::H);
      const cf ov = apply_ops(so, chan, mk(v.x, v.y), f1, kh, P::H);
      t0[q * P::T] = V(ou.x, ou.y);
      t1[q * P::T] = V(ov.x, ov.y);
    }
    TB_UNROLL
    for (int q = 0; q < P::Q1; ++q) {
      a[q] = t0[q * P::T];
      b[q] = t1[q * P::T];
    }
  }
  Dv<P::Q1, false>::run(a);
  Dv<P::Q1, false>::run(b);
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) {
    t0[q * P::T] = a[q] + b[q];
    t1[q * P::T] = a[q] - b[q];
  }
}

// stage-0 loads / stores of a split tile: column pair c of row j; columns c < TH from the first
// half (Sc + c), the others from the partner columns (Sc + nh + c - TH)
template <class P>
TB_HD int64_t split_col(int64_t nh, int c) {
  constexpr int TH = P::T / 2;
  return c < TH ? (int64_t)c : nh + (c - TH);
}
template <class P>
TB_HD void b_load_split(f4* r, const v2* __restrict__ Sc, int64_t ncols, int64_t nh, int it) {
  const int j = it / (P::T / 2), c = 2 * (it - j * (P::T / 2));
  const f4* s = reinterpret_cast<const f4*>(Sc + (int64_t)j * ncols + split_col<P>(nh, c));
  const int64_t st = (int64_t)P::L * (ncols / 2);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) r[q] = ld_stream<TB_NT_SPEC>(s + q * st);
}
template <class P>
TB_HD void b_s1_split(const v2* lds, v2* __restrict__ Sc, int64_t ncols, int64_t nh, int it) {
  const int j = it / (P::T / 2), c = 2 * (it - j * (P::T / 2));
  const v2* tw = lds + P::OFF_TW;
  const f4* t = reinterpret_cast<const f4*>(lds + j * P::T + c);
  v2 a[P::Q0], b[P::Q0];
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) {
    const f4 u = t[q * P::L * P::T / 2];
    a[q] = V(u.x, u.y);
    b[q] = V(u.z, u.w);
    if (q && j) {
      const v2 w = tw[j * q];
      a[q] = cmulc(a[q], w);
      b[q] = cmulc(b[q], w);
    }
  }
  Dv<P::Q0, false>::run(a);
  Dv<P::Q0, false>::run(b);
  f4* s = reinterpret_cast<f4*>(Sc + (int64_t)j * ncols + split_col<P>(nh, c));
  const int64_t st = (int64_t)P::L * (ncols / 2);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) s[q * st] = f4{a[q].x, a[q].y, b[q].x, b[q].y};
}

// H extents with a compile-time pass-B plan in the device library (tile width T = 16 columns)
#define TB_CT_TILE_H(X) X(240) X(128)
constexpr int kCtTileT = 16;
// paired (16-B lane) variant, used when the spectrum row length is even and divisible by it
constexpr int kCtTileT2 = 32;

}  // namespace ct
}  // namespace tb
