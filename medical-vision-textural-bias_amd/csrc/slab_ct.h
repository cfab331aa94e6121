// slab_ct.h -- compile-time-planned slab passes (A forward, C inverse) for the production shapes.
//
// The generic bodies in fft_core.h take every size, radix list and index map at run time.  For a
// slab shape fixed at compile time (BraTS C3: W = 240 = 16*15, D = 155 = 5*31; C2: 128 x 128) this
// header states the same transforms with every index map, loop trip count and twiddle position
// folded into constants, and with a dataflow that touches LDS fewer times, conflict-free:
//
//   pass A (per (bc, h) slab; x[w][d] real -> S[w'][kd] half spectrum)
//     F0  first D stage (radix R0, L = D/R0) straight from registers (the loads were issued while
//         the previous slab was transformed) -> pair rows Z[p][.] in LDS
//     D1  last D stage (radix R1, L = 1) in LDS
//     U   pair unpack Z -> X[kd][w] column image (read all -> barrier -> write all, via registers)
//     W0  first W stage (radix Q0, L = W/Q0) in LDS
//     W1  last W stage (radix Q1, L = 1): LDS -> registers -> HBM (S row pitch Dh, kd fastest)
//   pass C mirrors it: G0 (last inverse-W stage from registers) -> G1 -> R (repack) -> E1 -> E0
//   (the last inverse-D stage writes the real rows, scaled, with the min/max epilogue).
//
// Output layout and digit order are exactly those of the generic path (same radix preference as
// plan_host.h), so pass B and the op program are shared.  The host emulator (tests/emu) runs the
// same item functions serially.
//
// Reference being restated: Fourier.shift_fourier / inv_shift_fourier
// (source_code/filters_and_operators.py:594-632) -- see fft_core.h for the op mapping.
#pragma once

#include "fft_core.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define TB_UNROLL _Pragma("unroll")
#else
#define TB_UNROLL
#endif

namespace tb {
namespace ct {

// complex value as two scalar floats: the butterflies multiply by compile-time constants, which
// scalar v_fma_f32 / v_fmac_f32 take as literals (packed v_pk_fma_f32 would need every constant
// materialised in a register pair; the TU is built with -fno-slp-vectorize to keep it scalar)
struct alignas(8) v2 {
  float x, y;
};
TB_HD v2 V(float a, float b) { return v2{a, b}; }
TB_HD v2 operator+(v2 a, v2 b) { return v2{a.x + b.x, a.y + b.y}; }
TB_HD v2 operator-(v2 a, v2 b) { return v2{a.x - b.x, a.y - b.y}; }
TB_HD v2 operator*(float s, v2 a) { return v2{s * a.x, s * a.y}; }
TB_HD v2 operator*(v2 a, float s) { return v2{a.x * s, a.y * s}; }
TB_HD v2& operator+=(v2& a, v2 b) { a.x += b.x; a.y += b.y; return a; }
TB_HD v2 cmul(v2 a, v2 b) { return a.x * b + a.y * V(-b.y, b.x); }   // a * b
TB_HD v2 cmulc(v2 a, v2 b) { return b.x * a + b.y * V(a.y, -a.x); }  // a * conj(b)
TB_HD v2 conjv(v2 a) { return V(a.x, -a.y); }
template <bool FWD> TB_HD v2 rot(v2 a) { return FWD ? V(a.y, -a.x) : V(-a.y, a.x); }  // -i a | +i a

// ------------------------------------------------------------------ in-register DFTs (v2)
template <int R, bool FWD> struct Dv;

template <bool F> struct Dv<2, F> {
  TB_HD static void run(v2* a) { const v2 t = a[1]; a[1] = a[0] - t; a[0] = a[0] + t; }
};
template <bool F> struct Dv<3, F> {
  TB_HD static void run(v2* a) {
    const v2 t1 = a[1] + a[2], t2 = a[1] - a[2];
    const v2 m = a[0] - 0.5f * t1;
    const v2 r = rot<F>(0.86602540378443864676f * t2);
    a[0] = a[0] + t1;
    a[1] = m + r;
    a[2] = m - r;
  }
};
template <bool F> struct Dv<4, F> {
  TB_HD static void run(v2* a) {
    const v2 t0 = a[0] + a[2], t1 = a[0] - a[2];
    const v2 t2 = a[1] + a[3], t3 = rot<F>(a[1] - a[3]);
    a[0] = t0 + t2;
    a[2] = t0 - t2;
    a[1] = t1 + t3;
    a[3] = t1 - t3;
  }
};

// odd R: conjugate-pair symmetric direct DFT; st(k, y_k) receives each output as it is formed
template <int R, bool FWD, class Store>
TB_HD void dft_odd(v2* a, Store st) {
  constexpr int M = (R - 1) / 2;
  v2 y0 = a[0];
  TB_UNROLL
  for (int p = 1; p <= M; ++p) {
    const v2 s = a[p] + a[R - p], d = a[p] - a[R - p];
    a[p] = s;
    a[R - p] = d;
    y0 += s;
  }
  st(0, y0);
  TB_UNROLL
  for (int k = 1; k <= M; ++k) {
    v2 A = a[0], B = V(0.f, 0.f);
    TB_UNROLL
    for (int p = 1; p <= M; ++p) {
      const int m = (p * k) % R;
      A += Trig<R>::tab.c[m] * a[p];
      B += Trig<R>::tab.s[m] * a[R - p];
    }
    const v2 iB = V(-B.y, B.x);
    st(k, FWD ? A - iB : A + iB);
    st(R - k, FWD ? A + iB : A - iB);
  }
}
template <int R, bool F> struct DvOdd {
  TB_HD static void run(v2* a) {
    v2 o[R];
    dft_odd<R, F>(a, [&](int k, v2 v) { o[k] = v; });
    TB_UNROLL
    for (int k = 0; k < R; ++k) a[k] = o[k];
  }
};
template <bool F> struct Dv<5, F> : DvOdd<5, F> {};
template <bool F> struct Dv<7, F> : DvOdd<7, F> {};
template <bool F> struct Dv<11, F> : DvOdd<11, F> {};
template <bool F> struct Dv<13, F> : DvOdd<13, F> {};
template <bool F> struct Dv<17, F> : DvOdd<17, F> {};
template <bool F> struct Dv<19, F> : DvOdd<19, F> {};
template <bool F> struct Dv<23, F> : DvOdd<23, F> {};
template <bool F> struct Dv<29, F> : DvOdd<29, F> {};
template <bool F> struct Dv<31, F> : DvOdd<31, F> {};

// composite R = R1*R2 (Cooley-Tukey, constant twiddles): a[n1 + R1*n2] -> X[k2 + R2*k1]
template <int R1, int R2, bool F> struct DvComp {
  TB_HD static void run(v2* a) {
    constexpr int R = R1 * R2;
    v2 t[R];
    TB_UNROLL
    for (int n1 = 0; n1 < R1; ++n1) {
      v2 v[R2];
      TB_UNROLL
      for (int n2 = 0; n2 < R2; ++n2) v[n2] = a[n1 + R1 * n2];
      Dv<R2, F>::run(v);
      TB_UNROLL
      for (int k2 = 0; k2 < R2; ++k2) {
        const int m = (n1 * k2) % R;
        if (m == 0) {
          t[n1 + R1 * k2] = v[k2];
        } else {
          const float c = Trig<R>::tab.c[m];
          const float s = F ? -Trig<R>::tab.s[m] : Trig<R>::tab.s[m];
          t[n1 + R1 * k2] = cmul(v[k2], V(c, s));
        }
      }
    }
    TB_UNROLL
    for (int k2 = 0; k2 < R2; ++k2) {
      v2 v[R1];
      TB_UNROLL
      for (int n1 = 0; n1 < R1; ++n1) v[n1] = t[n1 + R1 * k2];
      Dv<R1, F>::run(v);
      TB_UNROLL
      for (int k1 = 0; k1 < R1; ++k1) a[k2 + R2 * k1] = v[k1];
    }
  }
};
template <bool F> struct Dv<6, F> : DvComp<2, 3, F> {};
template <bool F> struct Dv<8, F> : DvComp<2, 4, F> {};
template <bool F> struct Dv<9, F> : DvComp<3, 3, F> {};
template <bool F> struct Dv<10, F> : DvComp<2, 5, F> {};
template <bool F> struct Dv<12, F> : DvComp<4, 3, F> {};
template <bool F> struct Dv<15, F> : DvComp<3, 5, F> {};
template <bool F> struct Dv<16, F> : DvComp<4, 4, F> {};

template <int R> struct OddPrime {
  static constexpr bool value = (R == 5 || R == 7 || R == 11 || R == 13 || R == 17 || R == 19 || R == 23 ||
                                 R == 29 || R == 31);
};

// DFT of a[R] delivering outputs through st(k, v): streamed for odd primes (fewer live registers)
template <int R, bool F, class Store>
TB_HD void dft_store(v2* a, Store st) {
  if constexpr (OddPrime<R>::value) {
    dft_odd<R, F>(a, st);
  } else {
    Dv<R, F>::run(a);
    TB_UNROLL
    for (int q = 0; q < R; ++q) st(q, a[q]);
  }
}

// ------------------------------------------------------------------ compile-time plan
constexpr int kPref[] = {16, 15, 12, 10, 9, 8, 6, 5, 4, 3, 2, 7, 11, 13, 17, 19, 23, 29, 31};  // plan_host.h
constexpr int first_radix(int n) {
  for (int r : kPref)
    if (n % r == 0) return r;
  return 0;
}
// true when n factors (by the plan's preference order) into exactly two supported radices
constexpr bool two_stage(int n) {
  const int r0 = first_radix(n);
  return r0 > 1 && n / r0 > 1 && first_radix(n / r0) == n / r0;
}

// Slab shape W x D with two DIF stages per axis (D = R0*R1, W = Q0*Q1).
// LDS (complex units):  X[kd][w] column image, pitch PX = W+1 (odd: conflict-free column walks)
//                        | Z[p][d] pair rows, pitch D   (the same bytes, phases apart)
//                        then twW[W], twD[D].
template <int W_, int D_> struct SlabPlan {
  static constexpr int W = W_, D = D_, Dh = D / 2 + 1, NP = W / 2, PR = D;
  static constexpr int Dn = (D % 2 == 0) ? D / 2 : -1;
  static constexpr int R0 = first_radix(D), R1 = D / R0, L0 = R1;
  static constexpr int Q0 = first_radix(W), Q1 = W / Q0, LW = Q1;
  static_assert(two_stage(D), "D must factor as two supported radices");
  static_assert(two_stage(W), "W must factor as two supported radices");
  static_assert(W % 2 == 0, "pair rows need an even W");
  static constexpr int PX = W + 1;
  static constexpr int XCF = Dh * PX, ZCF = NP * PR;
  static constexpr int OFF_TWW = XCF > ZCF ? XCF : ZCF;
  static constexpr int OFF_TWD = OFF_TWW + W;
  static constexpr int TOTAL = OFF_TWD + D;
  static constexpr size_t LDS_BYTES = (size_t)TOTAL * 8;
  // work-item counts of the phases
  static constexpr int N_F0 = NP * L0;   // (p, j)    D stage 0  (pass C: E0)
  static constexpr int N_D1 = NP * R0;   // (p, blk)  D stage 1  (pass C: E1)
  static constexpr int N_U = NP * Dh;    // (p, kd)   pair unpack / repack
  static constexpr int N_W0 = Dh * LW;   // (kd, j)   W stage 0  (pass C: G1)
  static constexpr int N_W1 = Dh * Q0;   // (kd, blk) W stage 1  (pass C: G0)
  TB_HD static int rev(int k) { return (k % R0) * L0 + k / R0; }  // D frequency -> DIF slot
  // Fused D stage 1 + pair (un)pack (odd R0 and D): the stage-1 butterflies blk and R0 - blk hold
  // mirror frequencies (k = blk + R0 q and D - k = (R0 - blk) + R0 (R1 - 1 - q)), so one work item
  // per (p, group g) -- g = 0: butterfly 0 alone, g > 0: butterflies g and R0 - g -- owns every
  // (k, D - k) pair it needs and no unpack phase is required.
  static constexpr bool FUSED_DU = (R0 % 2 == 1) && (D % 2 == 1);
  static constexpr int G = R0 / 2 + 1;
  static constexpr int N_DU = NP * G;    // (g, p)   fused D stage 1 + unpack (pass C: repack + E1)
};

template <int N, int NT> struct Slots { static constexpr int value = (N + NT - 1) / NT; };

// ------------------------------------------------------------------ pass A phases
// F0 item (p, j): the R0 inputs of rows 2p and 2p+1 (re, im of the pair row), from global memory
template <class P>
TB_HD void a_load(v2* r, const float* __restrict__ xb, int64_t sw, int it) {
  const int p = it / P::L0, j = it - p * P::L0;
  const float* r0 = xb + (int64_t)(2 * p) * sw + j;
  const float* r1 = r0 + sw;
  TB_UNROLL
  for (int q = 0; q < P::R0; ++q) r[q] = V(r0[q * P::L0], r1[q * P::L0]);
}

// F0 inputs from the raw slab image staged in LDS (floats [w][d], pitch D: the same bytes as Z)
template <class P>
TB_HD void a_load_raw(const float* raw, v2* r, int it) {
  const int p = it / P::L0, j = it - p * P::L0;
  const float* r0 = raw + (2 * p) * P::D + j;
  const float* r1 = r0 + P::D;
  TB_UNROLL
  for (int q = 0; q < P::R0; ++q) r[q] = V(r0[q * P::L0], r1[q * P::L0]);
}

template <class P>
TB_HD void a_f0(v2* lds, const v2* r, int it) {
  const int p = it / P::L0, j = it - p * P::L0;
  const v2* tw = lds + P::OFF_TWD;
  v2 a[P::R0];
  TB_UNROLL
  for (int q = 0; q < P::R0; ++q) a[q] = r[q];
  Dv<P::R0, true>::run(a);
  v2* z = lds + p * P::PR + j;
  z[0] = a[0];
  TB_UNROLL
  for (int q = 1; q < P::R0; ++q) z[q * P::L0] = j ? cmul(a[q], tw[j * q]) : a[q];
}

template <class P>
TB_HD void a_d1(v2* lds, int it) {
  const int p = it / P::R0, blk = it - p * P::R0;
  v2* z = lds + p * P::PR + blk * P::L0;
  v2 a[P::R1];
  TB_UNROLL
  for (int q = 0; q < P::R1; ++q) a[q] = z[q];
  dft_store<P::R1, true>(a, [&](int q, v2 v) { z[q] = v; });
}

// U: read (p, kd) of the pair spectrum and split it into the two rows' spectra
template <class P>
TB_HD void a_u_read(const v2* lds, v2* r, int it) {
  const int p = it / P::Dh, k = it - p * P::Dh;
  const int m = k ? P::D - k : 0;
  const v2* z = lds + p * P::PR;
  const v2 zk = z[P::rev(k)], zm = conjv(z[P::rev(m)]);
  r[0] = 0.5f * (zk + zm);
  const v2 dd = 0.5f * (zk - zm);
  r[1] = V(dd.y, -dd.x);  // (zk - zm) / (2i)
}
template <class P>
TB_HD void a_u_write(v2* lds, const v2* r, int it) {
  const int p = it / P::Dh, k = it - p * P::Dh;
  v2* x = lds + k * P::PX + 2 * p;
  x[0] = r[0];
  x[1] = r[1];
}

// DU (fused D stage 1 + unpack), item (g, p) with p fastest: load the stage-1 inputs of butterflies
// g and R0 - g of pair row p into registers (r[0, R1) and r[R1, 2 R1)); after a barrier (X overlaps
// Z) a_du_compute transforms them and writes the two rows' spectra X[k][2p], X[k][2p + 1], k < Dh.
template <class P>
TB_HD void a_du_load(const v2* lds, v2* r, int it) {
  const int g = it / P::NP, p = it - g * P::NP;
  const v2* z = lds + p * P::PR;
  const int b2 = g ? P::R0 - g : 0;
  TB_UNROLL
  for (int q = 0; q < P::R1; ++q) r[q] = z[g * P::L0 + q];
  TB_UNROLL
  for (int q = 0; q < P::R1; ++q) r[P::R1 + q] = z[b2 * P::L0 + q];
}
// X[k][2p], X[k][2p+1] from Z(k) and Z(D - k): (zk + conj zm) / 2, (zk - conj zm) / (2i)
template <class P>
TB_HD void a_x_write(v2* lds, int k, int p, v2 zk, v2 zmk) {
  const v2 zm = conjv(zmk);
  v2* x = lds + k * P::PX + 2 * p;
  x[0] = 0.5f * (zk + zm);
  const v2 dd = 0.5f * (zk - zm);
  x[1] = V(dd.y, -dd.x);
}
template <class P>
TB_HD void a_du_compute(v2* lds, v2* r, int it) {
  static_assert(P::FUSED_DU, "fused DU needs odd R0 and D");
  const int g = it / P::NP, p = it - g * P::NP;
  v2 o1[P::R1];
  dft_store<P::R1, true>(r, [&](int q, v2 v) { o1[q] = v; });
  if (g == 0) {  // k = R0 q, mirror D - k = R0 (R1 - q)
    TB_UNROLL
    for (int q = 0; q < P::R1; ++q)
      if (P::R0 * q < P::Dh) a_x_write<P>(lds, P::R0 * q, p, o1[q], o1[(P::R1 - q) % P::R1]);
  } else {       // butterfly R0 - g streams its outputs; each pairs with o1[R1 - 1 - q]
    const int b2 = P::R0 - g;
    dft_store<P::R1, true>(r + P::R1, [&](int q, v2 v) {
      const int q1 = P::R1 - 1 - q;
      const int k2 = b2 + P::R0 * q, k1 = g + P::R0 * q1;  // k1 + k2 = D: exactly one is < Dh
      if (k2 < P::Dh) a_x_write<P>(lds, k2, p, v, o1[q1]);
      else a_x_write<P>(lds, k1, p, o1[q1], v);
    });
  }
}

template <class P>
TB_HD void a_w0(v2* lds, int it) {
  const int j = it / P::Dh, k = it - j * P::Dh;
  const v2* tw = lds + P::OFF_TWW;
  v2* x = lds + k * P::PX + j;
  v2 a[P::Q0];
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) a[q] = x[q * P::LW];
  Dv<P::Q0, true>::run(a);
  x[0] = a[0];
  TB_UNROLL
  for (int q = 1; q < P::Q0; ++q) x[q * P::LW] = j ? cmul(a[q], tw[j * q]) : a[q];
}

// W1: last W stage, results straight to the slab's half spectrum Sb[w'][kd]
template <class P>
TB_HD void a_w1(const v2* lds, v2* __restrict__ Sb, int it) {
  const int blk = it / P::Dh, k = it - blk * P::Dh;
  const v2* x = lds + k * P::PX + blk * P::LW;
  v2 a[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = x[q];
  v2* s = Sb + (blk * P::LW) * P::Dh + k;
  dft_store<P::Q1, true>(a, [&](int q, v2 v) { s[q * P::Dh] = v; });
}

// ------------------------------------------------------------------ pass C phases
// G0 item (kd, blk): the Q1 spectrum values of the first inverse-W butterfly, from global memory
template <class P>
TB_HD void c_load(v2* r, const v2* __restrict__ Sb, int it) {
  const int blk = it / P::Dh, k = it - blk * P::Dh;
  const v2* s = Sb + (blk * P::LW) * P::Dh + k;
  typedef float f2v __attribute__((ext_vector_type(2)));
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) {
    const f2v t = ld_stream<TB_NT_SPEC>(reinterpret_cast<const f2v*>(s + q * P::Dh));
    r[q] = V(t.x, t.y);
  }
}

template <class P>
TB_HD void c_g0(v2* lds, const v2* r, int it) {
  const int blk = it / P::Dh, k = it - blk * P::Dh;
  v2 a[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = r[q];
  v2* x = lds + k * P::PX + blk * P::LW;
  dft_store<P::Q1, false>(a, [&](int q, v2 v) { x[q] = v; });
}

template <class P>
TB_HD void c_g1(v2* lds, int it) {
  const int j = it / P::Dh, k = it - j * P::Dh;
  const v2* tw = lds + P::OFF_TWW;
  v2* x = lds + k * P::PX + j;
  v2 a[P::Q0];
  a[0] = x[0];
  TB_UNROLL
  for (int q = 1; q < P::Q0; ++q) a[q] = j ? cmulc(x[q * P::LW], tw[j * q]) : x[q * P::LW];
  Dv<P::Q0, false>::run(a);
  TB_UNROLL
  for (int q = 0; q < P::Q0; ++q) x[q * P::LW] = a[q];
}

// R: rows (2p, 2p+1) of column kd -> registers; then the pair spectrum slots of (p, kd)
template <class P>
TB_HD void c_r_read(const v2* lds, v2* r, int it) {
  const int p = it / P::Dh, k = it - p * P::Dh;
  const v2* x = lds + k * P::PX + 2 * p;
  r[0] = x[0];
  r[1] = x[1];
}
template <class P>
TB_HD void c_r_write(v2* lds, const v2* r, int it) {
  const int p = it / P::Dh, k = it - p * P::Dh;
  v2* z = lds + p * P::PR;
  const v2 xa = r[0], xb = r[1];
  if (k == 0 || k == P::Dn) {
    z[P::rev(k)] = V(xa.x, xb.x);  // c2r keeps Re of DC / Nyquist
  } else {
    z[P::rev(k)] = V(xa.x - xb.y, xa.y + xb.x);         // xa + i xb
    z[P::rev(P::D - k)] = V(xa.x + xb.y, xb.x - xa.y);  // conj(xa) + i conj(xb)
  }
}

// RE (fused repack + inverse D stage 1), item (g, p): gather the (k, D - k) pairs of butterflies
// g and R0 - g into their stage-1 inputs (registers); after a barrier (Z overlaps X) c_re_compute
// runs the inverse butterflies in place of pair row p.
template <class P>
TB_HD void c_re_load(const v2* lds, v2* r, int it) {
  const int g = it / P::NP, p = it - g * P::NP;
  if (g == 0) {
    TB_UNROLL
    for (int q = 0; q < P::R1; ++q) {
      if (P::R0 * q >= P::Dh) continue;
      const int k = P::R0 * q;
      const v2* x = lds + k * P::PX + 2 * p;
      const v2 xa = x[0], xb = x[1];
      if (k == 0) {
        r[0] = V(xa.x, xb.x);  // c2r keeps Re of DC
      } else {
        r[q] = V(xa.x - xb.y, xa.y + xb.x);                   // Z(k) = xa + i xb
        r[P::R1 - q] = V(xa.x + xb.y, xb.x - xa.y);           // Z(D - k) = conj(xa) + i conj(xb)
      }
    }
  } else {
    const int b2 = P::R0 - g;
    TB_UNROLL
    for (int q = 0; q < P::R1; ++q) {  // pair (k2 = b2 + R0 q, k1 = g + R0 (R1 - 1 - q))
      const int q1 = P::R1 - 1 - q;
      const int k2 = b2 + P::R0 * q, k1 = g + P::R0 * q1;
      const bool two = k2 < P::Dh;     // the stored (< Dh) member of the pair
      const v2* x = lds + (two ? k2 : k1) * P::PX + 2 * p;
      const v2 xa = x[0], xb = x[1];
      const v2 zs = V(xa.x - xb.y, xa.y + xb.x), zm = V(xa.x + xb.y, xb.x - xa.y);
      r[P::R1 + q] = two ? zs : zm;    // butterfly b2, output q  = Z(k2)
      r[q1] = two ? zm : zs;           // butterfly g,  output q1 = Z(k1)
    }
  }
}
template <class P>
TB_HD void c_re_compute(v2* lds, v2* r, int it) {
  static_assert(P::FUSED_DU, "fused RE needs odd R0 and D");
  const int g = it / P::NP, p = it - g * P::NP;
  v2* z = lds + p * P::PR;
  v2* z1 = z + g * P::L0;
  dft_store<P::R1, false>(r, [&](int q, v2 v) { z1[q] = v; });
  if (g != 0) {
    v2* z2 = z + (P::R0 - g) * P::L0;
    dft_store<P::R1, false>(r + P::R1, [&](int q, v2 v) { z2[q] = v; });
  }
}

template <class P>
TB_HD void c_e1(v2* lds, int it) {
  const int p = it / P::R0, blk = it - p * P::R0;
  v2* z = lds + p * P::PR + blk * P::L0;
  v2 a[P::R1];
  TB_UNROLL
  for (int q = 0; q < P::R1; ++q) a[q] = z[q];
  dft_store<P::R1, false>(a, [&](int q, v2 v) { z[q] = v; });
}

// E0: last inverse D stage; outputs d = j + L0*q of rows 2p (re) and 2p+1 (im), scaled
template <class P>
TB_HD void c_e0(const v2* lds, float* __restrict__ yb, int64_t sw, float scale, int it, float& lo, float& hi) {
  const int p = it / P::L0, j = it - p * P::L0;
  const v2* tw = lds + P::OFF_TWD;
  const v2* z = lds + p * P::PR + j;
  v2 a[P::R0];
  a[0] = z[0];
  TB_UNROLL
  for (int q = 1; q < P::R0; ++q) a[q] = j ? cmulc(z[q * P::L0], tw[j * q]) : z[q * P::L0];
  Dv<P::R0, false>::run(a);
  float* r0 = yb + (int64_t)(2 * p) * sw + j;
  float* r1 = r0 + sw;
  TB_UNROLL
  for (int q = 0; q < P::R0; ++q) {
    const v2 v = a[q] * scale;
    st_stream<TB_NT_STORES>(r0 + q * P::L0, v.x);
    st_stream<TB_NT_STORES>(r1 + q * P::L0, v.y);
    lo = v.x < lo ? v.x : lo;
    hi = v.x > hi ? v.x : hi;
    lo = v.y < lo ? v.y : lo;
    hi = v.y > hi ? v.y : hi;
  }
}

// twiddle tables into LDS (from the plan's device tables)
template <class P, class Ctx>
TB_HD void load_tw(Ctx& ctx, v2* lds, const tb_plan_dev& pl) {
  for (int i = ctx.tid; i < P::W; i += ctx.nthreads) lds[P::OFF_TWW + i] = V(pl.tw[1][i].x, pl.tw[1][i].y);
  for (int i = ctx.tid; i < P::D; i += ctx.nthreads) lds[P::OFF_TWD + i] = V(pl.tw[2][i].x, pl.tw[2][i].y);
}

// ------------------------------------------------------------------ half slabs (W split by parity)
// A (bc, h) slab's W transform split at its last radix-2 step (decimation in time): unit (slab, e)
// transforms rows w = 2 w'' + e (w'' < W/2) with the SlabPlan<W/2, D> item functions -- R2C along D,
// the W/2-point DFT along w'' -- and for e = 1 scales the result by w^k'' (w = e^{-2 pi i / W}).  The
// half spectrum is then stored "split": row w' = e W/2 + slot(k'') of the slab holds E0(k'') (e = 0)
// or w^k'' E1(k'') (e = 1), and pass B finishes the W transform with the butterfly
// X(k'') = E0 + T1, X(k'' + W/2) = E0 - T1 (and stores X' (k'') +- X' (k'' + W/2) back).  Pass C
// inverts: unit (slab, e) reads its rows, scales e = 1 by w^-k'', runs the inverse W/2-point DFT and
// the C2R D transform, and writes rows 2 w'' + e.  Each unit needs half the LDS of a slab, so two
// workgroups share a CU and one's HBM traffic overlaps the other's butterflies (a whole slab fills a
// CU's LDS: its loads and stores stall the CU's only workgroup).
template <int W_, int D_> struct HalfPlan {
  using P = SlabPlan<W_ / 2, D_>;
  static constexpr int W = W_, W2 = W_ / 2, D = D_, Dh = P::Dh;
  static_assert(W_ % 2 == 0, "even W");
  static constexpr int OFF_TWE = P::TOTAL;  // w^k, k < W/2 (the W-point table)
  static constexpr int TOTAL = OFF_TWE + W2;
  static constexpr size_t LDS_BYTES = (size_t)TOTAL * 8;
  static constexpr int NRAW = W2 * D;  // raw floats of a unit (pass A staging, the bytes of Z)
  TB_HD static int freq(int slot) { return (slot / P::LW) + P::Q0 * (slot % P::LW); }  // slot -> k''
};

// twiddles of a half unit: the W/2-point table (even entries of the W-point one), D, and w^k
template <class HP, class Ctx>
TB_HD void load_tw_half(Ctx& ctx, v2* lds, const tb_plan_dev& pl) {
  using P = typename HP::P;
  for (int i = ctx.tid; i < HP::W2; i += ctx.nthreads) {
    lds[P::OFF_TWW + i] = V(pl.tw[1][2 * i].x, pl.tw[1][2 * i].y);
    lds[HP::OFF_TWE + i] = V(pl.tw[1][i].x, pl.tw[1][i].y);
  }
  for (int i = ctx.tid; i < P::D; i += ctx.nthreads) lds[P::OFF_TWD + i] = V(pl.tw[2][i].x, pl.tw[2][i].y);
}

// W1 of a half unit: slot blk*LW + q holds k'' = blk + Q0 q; e = 1 scales by w^k''
template <class HP>
TB_HD void a_w1_half(const v2* lds, v2* __restrict__ Sb, int e, int it) {
  using P = typename HP::P;
  const int blk = it / P::Dh, k = it - blk * P::Dh;
  const v2* x = lds + k * P::PX + blk * P::LW;
  const v2* te = lds + HP::OFF_TWE;
  v2 a[P::Q1];
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) a[q] = x[q];
  v2* s = Sb + (blk * P::LW) * P::Dh + k;
  dft_store<P::Q1, true>(a, [&](int q, v2 v) { s[q * P::Dh] = e ? cmul(v, te[blk + P::Q0 * q]) : v; });
}

// G0 inputs of a half unit (pass C): slot blk*LW + q of the unit's rows, e = 1 scaled by w^-k''
template <class HP>
TB_HD void c_load_half(v2* r, const v2* __restrict__ Sb, int it) {
  using P = typename HP::P;
  const int blk = it / P::Dh, k = it - blk * P::Dh;
  const v2* s = Sb + (blk * P::LW) * P::Dh + k;
  typedef float f2v __attribute__((ext_vector_type(2)));
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) {
    const f2v t = ld_stream<TB_NT_SPEC>(reinterpret_cast<const f2v*>(s + q * P::Dh));
    r[q] = V(t.x, t.y);
  }
}
template <class HP>
TB_HD void c_twiddle_half(const v2* lds, v2* r, int e, int it) {
  using P = typename HP::P;
  if (!e) return;
  const int blk = it / P::Dh;
  const v2* te = lds + HP::OFF_TWE;
  TB_UNROLL
  for (int q = 0; q < P::Q1; ++q) r[q] = cmulc(r[q], te[blk + P::Q0 * q]);
}

// Slab shapes (W, D) whose whole-slab passes have a compile-time plan in the device library
#define TB_CT_SLAB_SHAPES(X) X(128, 128) X(128, 64)
// Slab shapes that run as half units (split spectrum; W/2 two-stage, half slab <= 80 KB of LDS).  Their
// whole-slab compiled kernels were dropped in round 6 (a 150 KB slab per CU spilled 104-400 B/lane and ran
// 1.3x slower than the half units): with half units off they take the run-time-planned passes.
#define TB_CT_HALF_SHAPES(X) X(240, 155)

}  // namespace ct
}  // namespace tb
