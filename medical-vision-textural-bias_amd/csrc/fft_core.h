// fft_core.h -- the per-workgroup bodies of the texbias k-space filter passes.
//
// Shared by the gfx950 kernels (texbias.hip) and by the serial host emulator
// used ONLY by the CPU test-suite (tests/emu/emu.cpp).  Every body is written
// as barrier-separated phases; inside a phase the work items are independent
// (each in-place butterfly owns its r LDS slots), so the emulator runs a block
// with one "thread" and a no-op barrier and computes bit-for-bit the same
// schedule of arithmetic per element.
//
// Reference being restated (file:line under /root/reference):
//   Fourier.shift_fourier / inv_shift_fourier   source_code/filters_and_operators.py:594-632
//   disk_mask                                    source_code/filters_and_operators.py:105-206
//   RandPlaneWaves_ellipsoid                     source_code/filters_and_operators.py:370-414
//   WrapArtifact                                 source_code/filters_and_operators.py:503-515
//   GibbsNoise._apply_mask                       source_code/filters_and_operators.py:678-705
//   KSpaceSpikeNoise                             source_code/filters_and_operators.py:906-983
//   GibbsNoiseLayer._apply_mask                  source_code/stylization_layers.py:91-116
//
// Transform layout (DESIGN.md "Data layout in HBM"):
//   image   x[bc][h][w][d]   float32, d contiguous (D = last spatial axis)
//   spectrum S[bc][h][w'][kd] complex64, kd in [0, D/2]  (real-input half spectrum)
//     h and w' are in DIGIT-REVERSED order (in-place mixed-radix DIF output);
//     the inverse DIT consumes that order directly, so no permutation pass exists.
#pragma once

#include <stdint.h>
#include "texbias.h"

#if defined(__HIPCC__)
#define TB_HD __host__ __device__ __forceinline__
#define TB_HD_NOINLINE __host__ __device__ __attribute__((noinline))
#else
#define TB_HD inline
#define TB_HD_NOINLINE __attribute__((noinline))
#endif

#define TB_MAX_STAGES 8

// Loads of data a kernel reads once are nontemporal: a nontemporal read does not allocate in the
// Infinity Cache, so one that follows a large write does not evict the written dirty lines and pay
// their write-back (scripts/micro/read_bw.hip, 285.7 MB right after a 294 MB write: 86 us with plain
// 16-B loads, 48 us nontemporal; 42-46 us both after a read).  TB_NT_LOADS: image reads (point,
// wrap and slab forward passes); TB_NT_SPEC: the full route's spectrum reads (passes B and C).
#ifndef TB_NT_LOADS
#define TB_NT_LOADS 1
#endif
#ifndef TB_NT_SPEC
#define TB_NT_SPEC 1
#endif
#ifndef TB_NT_WRAP  // the separable wrap pass (measured separately: it reads the clean input)
#define TB_NT_WRAP 0
#endif
template <bool NT, class T>
TB_HD T ld_stream(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (NT) return __builtin_nontemporal_load(p);
#endif
  return *p;
}
// TB_NT_STORES: the filtered image's stores nontemporal as well (point apply, wrap, slab inverse)
#ifndef TB_NT_STORES
#define TB_NT_STORES 0
#endif
template <bool NT, class T>
TB_HD void st_stream(T* p, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (NT) {
    __builtin_nontemporal_store(v, p);
    return;
  }
#endif
  *p = v;
}
typedef float tb_f4v __attribute__((ext_vector_type(4)));

namespace tb {

struct alignas(8) cf {
  float x, y;
};

// one FFT axis: length and its in-place DIF stage radices
struct tb_axis {
  int n, nst;
  int radix[TB_MAX_STAGES];
};

// device-visible plan (passed by value in the launch arguments)
struct tb_plan_dev {
  int H, W, D, pad;
  tb_axis ax[3];        // 0 = H, 1 = W, 2 = D
  const cf* tw[3];      // tw[a][t] = exp(-2 pi i t / n_a)
  const int* rev_d;     // D: frequency -> DIF slot
  const int* irev_h;    // H: DIF slot -> frequency
  const int* irev_w;    // W: DIF slot -> frequency
};

TB_HD cf mk(float a, float b) { cf r; r.x = a; r.y = b; return r; }
TB_HD cf add(cf a, cf b) { return mk(a.x + b.x, a.y + b.y); }
TB_HD cf sub(cf a, cf b) { return mk(a.x - b.x, a.y - b.y); }
TB_HD cf mul(cf a, cf b) { return mk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
TB_HD cf mulc(cf a, cf b) { return mk(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y); }  // a * conj(b)
TB_HD cf conj(cf a) { return mk(a.x, -a.y); }
TB_HD cf scl(cf a, float s) { return mk(a.x * s, a.y * s); }
// multiply by -i (forward) or +i (inverse)
template <bool FWD> TB_HD cf rot90(cf a) { return FWD ? mk(a.y, -a.x) : mk(-a.y, a.x); }

// ---------------------------------------------------------------- constants
// constexpr trig (compile-time butterfly constants for the odd-prime radices)
constexpr double kPi = 3.14159265358979323846264338327950288;
constexpr double csin_series(double x) {
  double term = x, sum = x;
  for (int i = 1; i < 30; ++i) { term *= -x * x / ((2 * i) * (2 * i + 1)); sum += term; }
  return sum;
}
constexpr double cred(double x) {  // reduce to [-pi, pi]
  while (x > kPi) x -= 2 * kPi;
  while (x < -kPi) x += 2 * kPi;
  return x;
}
constexpr double csin(double x) { return csin_series(cred(x)); }
constexpr double ccos(double x) { return csin(x + kPi / 2); }
// cos/sin(2 pi m / R) as a constexpr table: indexed with unrolled (constant) m the values
// fold into literals -- a direct constexpr call is NOT folded by hipcc for large R.
template <int R> struct TrigTab {
  float c[R], s[R];
  constexpr TrigTab() : c(), s() {
    for (int m = 0; m < R; ++m) {
      c[m] = (float)ccos(2.0 * kPi * m / R);
      s[m] = (float)csin(2.0 * kPi * m / R);
    }
  }
};
template <int R> struct Trig { static constexpr TrigTab<R> tab{}; };

// ------------------------------------------------------------- small DFTs
// In-register DFT of size R.  FWD: X[k] = sum_p a[p] e^{-2 pi i pk/R};
// inverse (unnormalised) uses e^{+...}.
template <int R, bool FWD> struct Dft;

template <bool FWD> struct Dft<2, FWD> {
  TB_HD static void run(cf* a) { cf t = a[1]; a[1] = sub(a[0], t); a[0] = add(a[0], t); }
};

template <bool FWD> struct Dft<3, FWD> {
  TB_HD static void run(cf* a) {
    const float c = -0.5f, s = 0.86602540378443864676f;
    cf t1 = add(a[1], a[2]), t2 = sub(a[1], a[2]);
    cf m = add(a[0], scl(t1, c));
    cf r = rot90<FWD>(scl(t2, s));  // -i*s*(a1-a2) forward
    a[0] = add(a[0], t1);
    a[1] = add(m, r);
    a[2] = sub(m, r);
  }
};

template <bool FWD> struct Dft<4, FWD> {
  TB_HD static void run(cf* a) {
    cf t0 = add(a[0], a[2]), t1 = sub(a[0], a[2]);
    cf t2 = add(a[1], a[3]), t3 = rot90<FWD>(sub(a[1], a[3]));
    a[0] = add(t0, t2);
    a[2] = sub(t0, t2);
    a[1] = add(t1, t3);
    a[3] = sub(t1, t3);
  }
};

// generic odd prime: conjugate-pair symmetric direct DFT (R-1)^2/4 complex*real pairs
template <int R, bool FWD> struct DftOdd {
  TB_HD static void run(cf* a) {
    constexpr int M = (R - 1) / 2;
    cf s[M + 1], d[M + 1];
    cf y0 = a[0];
#pragma unroll
    for (int p = 1; p <= M; ++p) {
      s[p] = add(a[p], a[R - p]);
      d[p] = sub(a[p], a[R - p]);
      y0 = add(y0, s[p]);
    }
    cf out[R];
    out[0] = y0;
#pragma unroll
    for (int k = 1; k <= M; ++k) {
      cf A = a[0], B = mk(0.f, 0.f);
#pragma unroll
      for (int p = 1; p <= M; ++p) {
        const int m = (p * k) % R;
        const float c = Trig<R>::tab.c[m];
        const float sn = Trig<R>::tab.s[m];
        A.x += s[p].x * c; A.y += s[p].y * c;
        B.x += d[p].x * sn; B.y += d[p].y * sn;
      }
      // forward: y[k] = A - i B, y[R-k] = A + i B ; inverse: swapped
      cf iB = mk(-B.y, B.x);
      out[k] = FWD ? sub(A, iB) : add(A, iB);
      out[R - k] = FWD ? add(A, iB) : sub(A, iB);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) a[k] = out[k];
  }
};
template <bool FWD> struct Dft<5, FWD> : DftOdd<5, FWD> {};
template <bool FWD> struct Dft<7, FWD> : DftOdd<7, FWD> {};
template <bool FWD> struct Dft<11, FWD> : DftOdd<11, FWD> {};
template <bool FWD> struct Dft<13, FWD> : DftOdd<13, FWD> {};
template <bool FWD> struct Dft<17, FWD> : DftOdd<17, FWD> {};
template <bool FWD> struct Dft<19, FWD> : DftOdd<19, FWD> {};
template <bool FWD> struct Dft<23, FWD> : DftOdd<23, FWD> {};
template <bool FWD> struct Dft<29, FWD> : DftOdd<29, FWD> {};
template <bool FWD> struct Dft<31, FWD> : DftOdd<31, FWD> {};

// composite R = R1*R2 in registers (Cooley-Tukey, constant twiddles):
// a[n1 + R1*n2] -> X[k2 + R2*k1]
template <int R1, int R2, bool FWD> struct DftComp {
  TB_HD static void run(cf* a) {
    constexpr int R = R1 * R2;
    cf t[R];
    // R1 DFTs of size R2 over n2 for each n1
#pragma unroll
    for (int n1 = 0; n1 < R1; ++n1) {
      cf v[R2];
#pragma unroll
      for (int n2 = 0; n2 < R2; ++n2) v[n2] = a[n1 + R1 * n2];
      Dft<R2, FWD>::run(v);
#pragma unroll
      for (int k2 = 0; k2 < R2; ++k2) {
        const int m = (n1 * k2) % R;
        if (m == 0) {
          t[n1 + R1 * k2] = v[k2];
        } else {
          const float c = Trig<R>::tab.c[m];
          const float sn = FWD ? -Trig<R>::tab.s[m] : Trig<R>::tab.s[m];
          t[n1 + R1 * k2] = mul(v[k2], mk(c, sn));
        }
      }
    }
    // R2 DFTs of size R1 over n1 for each k2
#pragma unroll
    for (int k2 = 0; k2 < R2; ++k2) {
      cf v[R1];
#pragma unroll
      for (int n1 = 0; n1 < R1; ++n1) v[n1] = t[n1 + R1 * k2];
      Dft<R1, FWD>::run(v);
#pragma unroll
      for (int k1 = 0; k1 < R1; ++k1) a[k2 + R2 * k1] = v[k1];
    }
  }
};
template <bool FWD> struct Dft<8, FWD> : DftComp<2, 4, FWD> {};
template <bool FWD> struct Dft<16, FWD> : DftComp<4, 4, FWD> {};
template <bool FWD> struct Dft<6, FWD> : DftComp<2, 3, FWD> {};
template <bool FWD> struct Dft<9, FWD> : DftComp<3, 3, FWD> {};
template <bool FWD> struct Dft<10, FWD> : DftComp<2, 5, FWD> {};
template <bool FWD> struct Dft<12, FWD> : DftComp<4, 3, FWD> {};
template <bool FWD> struct Dft<15, FWD> : DftComp<3, 5, FWD> {};

// ------------------------------------------------------------ integer helpers
// Division by a runtime-constant divisor for 0 <= t < 2^22: one float multiply + one correction
// (the exact integer division sequence costs ~25 VALU ops; it sits in every work loop).
struct FastDiv {
  int d;
  float inv;
  TB_HD static FastDiv make(int dv) { FastDiv f; f.d = dv > 0 ? dv : 1; f.inv = 1.0f / (float)f.d; return f; }
  TB_HD int div(int t) const {
    int q = (int)((float)t * inv);
    const int r = t - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return q;
  }
};

// ------------------------------------------------------------ batched copies
// Global <-> LDS copies issue U independent loads per thread before their first use, so a
// workgroup keeps U * nthreads requests in flight instead of waiting out HBM latency per element.
template <int U, class Ctx, class LoadF, class StoreF>
TB_HD void copy_batched(Ctx& ctx, int n, LoadF ld, StoreF st) {
  for (int b0 = ctx.tid; b0 < n; b0 += ctx.nthreads * U) {
    cf v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = b0 + u * ctx.nthreads;
      if (t < n) v[u] = ld(t);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = b0 + u * ctx.nthreads;
      if (t < n) st(t, v[u]);
    }
  }
}
constexpr int kCopyUnroll = 8;

// ------------------------------------------------------------ addressing
// pen(p) binds pencil p once per butterfly; pen(i) is then one multiply-add per element.
struct RowAddr {  // pair pencils along D: element d of pair p at p*PR + d
  int PR;
  struct Pen {
    int b;
    TB_HD int operator()(int i) const { return b + i; }
  };
  TB_HD Pen pen(int p) const { return Pen{p * PR}; }
};
struct TileAddr {  // H pencils of the pass-B tile: element h of column c at h*T + c
  int T;
  struct Pen {
    int c, T;
    TB_HD int operator()(int h) const { return h * T + c; }
  };
  TB_HD Pen pen(int c) const { return Pen{c, T}; }
};

// Accessors: acc.pen(p) -> {ld(i), st(i, v)} for element i of pencil p.  A stage reads through
// one accessor and writes through another, so the first stage of an axis can read HBM straight
// into registers and the last can write HBM from registers (no staging round trip through LDS).
template <class AddrF>
struct LdsAcc {
  cf* lds;
  AddrF addr;
  struct Pen {
    cf* lds;
    typename AddrF::Pen a;
    TB_HD cf ld(int i) const { return lds[a(i)]; }
    TB_HD void st(int i, cf v) const { lds[a(i)] = v; }
  };
  TB_HD Pen pen(int p) const { return Pen{lds, addr.pen(p)}; }
};
template <class AddrF>
TB_HD LdsAcc<AddrF> lds_acc(cf* lds, AddrF a) { return LdsAcc<AddrF>{lds, a}; }

struct StridedAcc {  // pencil p: base + p * pstride, element stride estride (complex, global)
  cf* base;
  int64_t pstride, estride;
  struct Pen {
    cf* b;
    int64_t es;
    TB_HD cf ld(int i) const { return b[i * es]; }
    TB_HD void st(int i, cf v) const { b[i * es] = v; }
  };
  TB_HD Pen pen(int p) const { return Pen{base + p * pstride, estride}; }
};

// ------------------------------------------------------ in-place stages
// Mixed-radix in-place DIF (Sande-Tukey).  Stage s (radix r, block length Lb,
// P = n/Lb = product of previous radices, L = Lb/r):
//   butterfly (blk, j): positions blk*Lb + j + q*L, q < r
//   y = DFT_r(x);  y[q] *= w_n^{j*q*P}
// After all stages position  sum_s q_s * L_s  holds X[q_1 + r_1 (q_2 + r_2 (...))].
// The inverse DIT runs the stages in reverse order with conj twiddles first.

// odd-prime butterfly that stores each output pair as soon as it is formed (keeps ~R+8 live
// complex registers instead of ~3R for the radix-31 stage of D = 155)
template <int R, bool FWD, class Store>
TB_HD void dft_odd_stream(cf* a, Store st) {
  constexpr int M = (R - 1) / 2;
  cf y0 = a[0];
#pragma unroll
  for (int p = 1; p <= M; ++p) {
    const cf s = add(a[p], a[R - p]), d = sub(a[p], a[R - p]);
    a[p] = s;
    a[R - p] = d;
    y0 = add(y0, s);
  }
  st(0, y0);
#pragma unroll
  for (int k = 1; k <= M; ++k) {
    cf A = a[0], B = mk(0.f, 0.f);
#pragma unroll
    for (int p = 1; p <= M; ++p) {
      const int m = (p * k) % R;
      const float c = Trig<R>::tab.c[m], sn = Trig<R>::tab.s[m];
      A.x += a[p].x * c; A.y += a[p].y * c;
      B.x += a[R - p].x * sn; B.y += a[R - p].y * sn;
    }
    const cf iB = mk(-B.y, B.x);
    st(k, FWD ? sub(A, iB) : add(A, iB));
    st(R - k, FWD ? add(A, iB) : sub(A, iB));
  }
}

// the streamed symmetric form is used for the odd primes >= 11 only (composites go through DftComp)
template <int R> struct IsStreamed {
  static constexpr bool value = (R == 11 || R == 13 || R == 17 || R == 19 || R == 23 || R == 29 || R == 31);
};

struct StageGeo {  // butterfly -> (pencil, base position) for one stage
  int L, Lb, npen, nb;
  FastDiv dpen, dnb, dL;
  bool pencil_fast;
  TB_HD static StageGeo make(int R, int Lb, int npen, int n, bool pf) {
    StageGeo g;
    g.Lb = Lb;
    g.L = Lb / R;
    g.npen = npen;
    g.nb = n / R;
    g.dpen = FastDiv::make(npen);
    g.dnb = FastDiv::make(g.nb);
    g.dL = FastDiv::make(g.L);
    g.pencil_fast = pf;
    return g;
  }
  TB_HD void map(int t, int& p, int& base, int& j) const {
    int u;
    if (pencil_fast) { u = dpen.div(t); p = t - u * npen; }
    else { p = dnb.div(t); u = t - p * nb; }
    const int blk = dL.div(u);
    j = u - blk * L;
    base = blk * Lb + j;
  }
};

template <class Ctx, int R, bool FWD, class Src, class Dst>
TB_HD void stage_r(Ctx& ctx, Src src, Dst dst, const cf* tw, int Lb, int P, int npen, int n, bool pencil_fast) {
  const StageGeo g = StageGeo::make(R, Lb, npen, n, pencil_fast);
  const int L = g.L;
  const int total = npen * g.nb;
  for (int t = ctx.tid; t < total; t += ctx.nthreads) {
    int p, base, j;
    g.map(t, p, base, j);
    const auto sp = src.pen(p);
    const auto dp = dst.pen(p);
    cf a[R];
#pragma unroll
    for (int q = 0; q < R; ++q) a[q] = sp.ld(base + q * L);
    if constexpr (IsStreamed<R>::value) {
      if (!FWD && j) {
#pragma unroll
        for (int q = 1; q < R; ++q) a[q] = mulc(a[q], tw[j * q * P]);
      }
      dft_odd_stream<R, FWD>(a, [&](int q, cf v) {
        if (FWD && j && q) v = mul(v, tw[j * q * P]);
        dp.st(base + q * L, v);
      });
    } else {
      if (FWD) {
        Dft<R, true>::run(a);
        if (j) {
#pragma unroll
          for (int q = 1; q < R; ++q) a[q] = mul(a[q], tw[j * q * P]);
        }
      } else {
        if (j) {
#pragma unroll
          for (int q = 1; q < R; ++q) a[q] = mulc(a[q], tw[j * q * P]);
        }
        Dft<R, false>::run(a);
      }
#pragma unroll
      for (int q = 0; q < R; ++q) dp.st(base + q * L, a[q]);
    }
  }
}

// the op program called out of line: the large odd-prime butterflies would otherwise inline R
// copies of it (compile time and code size; those radices are rare on the H axis)
template <class OpsF, class CC>
TB_HD_NOINLINE cf ops_call(const OpsF& ops, const CC& cc, int pos, cf v) {
  return ops(cc, pos, v);
}

// last forward stage + per-coefficient ops + first inverse stage, in registers.  The last DIF
// stage has L = 1 and j = 0 (no twiddles): its butterfly groups are exactly the groups of the
// first DIT stage, so forward DFT -> ops(position) -> inverse DFT never leaves the thread.
template <class Ctx, int R, class Src, class Dst, class OpsF>
TB_HD void stage_mid_r(Ctx& ctx, Src src, Dst dst, int npen, int n, OpsF ops, bool pencil_fast) {
  const StageGeo g = StageGeo::make(R, R, npen, n, pencil_fast);
  const int total = npen * g.nb;
  for (int t = ctx.tid; t < total; t += ctx.nthreads) {
    int p, base, j;
    g.map(t, p, base, j);
    const auto sp = src.pen(p);
    const auto dp = dst.pen(p);
    cf a[R];
#pragma unroll
    for (int q = 0; q < R; ++q) a[q] = sp.ld(base + q);
    Dft<R, true>::run(a);
    const auto cc = ops.col(p);   // geometry shared by the butterfly's R coefficients
#pragma unroll
    for (int q = 0; q < R; ++q) {
      if constexpr (IsStreamed<R>::value) a[q] = ops_call(ops, cc, base + q, a[q]);  // one out-of-line copy
      else a[q] = ops(cc, base + q, a[q]);
    }
    Dft<R, false>::run(a);
#pragma unroll
    for (int q = 0; q < R; ++q) dp.st(base + q, a[q]);
  }
}

// Radix sets compiled into a kernel: RS 0 = {2..10, 12, 15, 16} (small register
// footprint), RS 1 adds the primes 11..31 (needed e.g. for D = 155 = 5 * 31).
#define TB_SMALL_RADICES(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(12) X(15) X(16)
#define TB_PRIME_RADICES(X) X(11) X(13) X(17) X(19) X(23) X(29) X(31)

template <class Ctx, bool FWD, int RS, class Src, class Dst>
TB_HD void stage(Ctx& ctx, Src src, Dst dst, const cf* tw, int r, int Lb, int P, int npen, int n, bool pf) {
#define TB_CASE(R) case R: stage_r<Ctx, R, FWD>(ctx, src, dst, tw, Lb, P, npen, n, pf); return;
  switch (r) { TB_SMALL_RADICES(TB_CASE) default: break; }
  if constexpr (RS == 1) {
    switch (r) { TB_PRIME_RADICES(TB_CASE) default: break; }
  }
#undef TB_CASE
}

template <class Ctx, int RS, class Src, class Dst, class OpsF>
TB_HD void stage_mid(Ctx& ctx, Src src, Dst dst, int r, int npen, int n, OpsF ops, bool pf) {
#define TB_CASE(R) case R: stage_mid_r<Ctx, R>(ctx, src, dst, npen, n, ops, pf); return;
  switch (r) { TB_SMALL_RADICES(TB_CASE) default: break; }
  if constexpr (RS == 1) {
    switch (r) { TB_PRIME_RADICES(TB_CASE) default: break; }
  }
#undef TB_CASE
}

TB_HD int prefix_product(const tb_axis& ax, int s) {
  int P = 1;
  for (int i = 0; i < s; ++i) P *= ax.radix[i];
  return P;
}

// forward DIF stages [s0, s1) in place through `acc`, a barrier after each
template <class Ctx, int RS, class Acc>
TB_HD void dif_stages(Ctx& ctx, Acc acc, const cf* tw, const tb_axis& ax, int s0, int s1, int npen, bool pf) {
  int P = prefix_product(ax, s0);
  for (int s = s0; s < s1; ++s) {
    const int r = ax.radix[s];
    stage<Ctx, true, RS>(ctx, acc, acc, tw, r, ax.n / P, P, npen, ax.n, pf);
    ctx.sync();
    P *= r;
  }
}

// inverse DIT stages s1-1 down to s0 in place through `acc`, a barrier after each
template <class Ctx, int RS, class Acc>
TB_HD void dit_stages(Ctx& ctx, Acc acc, const cf* tw, const tb_axis& ax, int s0, int s1, int npen, bool pf) {
  int P = prefix_product(ax, s1);
  for (int s = s1 - 1; s >= s0; --s) {
    const int r = ax.radix[s];
    P /= r;
    stage<Ctx, false, RS>(ctx, acc, acc, tw, r, ax.n / P, P, npen, ax.n, pf);
    ctx.sync();
  }
}

// whole-axis transforms through one accessor (used by the stats kernel and the tests)
template <class Ctx, int RS, class AddrF>
TB_HD void fft_dif(Ctx& ctx, cf* lds, const cf* tw, const tb_axis& ax, int npen, AddrF addr, bool pf) {
  dif_stages<Ctx, RS>(ctx, lds_acc(lds, addr), tw, ax, 0, ax.nst, npen, pf);
}
template <class Ctx, int RS, class AddrF>
TB_HD void fft_dit(Ctx& ctx, cf* lds, const cf* tw, const tb_axis& ax, int npen, AddrF addr, bool pf) {
  dit_stages<Ctx, RS>(ctx, lds_acc(lds, addr), tw, ax, 0, ax.nst, npen, pf);
}

// ------------------------------------------------------------- k-space ops
// Frequency bookkeeping per axis: unshifted index k in [0,n); the reference's
// fftshift-ed index is s = (k + n/2) mod n (n/2 floored).
TB_HD int shifted(int k, int n) { int s = k + n / 2; return s >= n ? s - n : s; }
TB_HD int negk(int k, int n) { return k == 0 ? 0 : n - k; }

// correctly rounded IEEE float32 division / square root (bit-exact mask geometry)
TB_HD float f32_div(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __fdiv_rn(a, b);
#else
  return a / b;
#endif
}
TB_HD float f32_sqrt(float a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __fsqrt_rn(a);
#else
  return __builtin_sqrtf(a);
#endif
}

// Per-axis geometry of a coefficient f (and its mirror -f), the only quantities the masks need:
//   dsq = (s - n/2)^2               disk_mask: centre floor(n/2) (filters_and_operators.py:176-187)
//   ef, en = (2s - (n-1))^2 at f, -f   GibbsNoise / GibbsNoiseLayer: 4*(s - (n-1)/2)^2, exact (:689-698)
//   odd = s & 1                      WrapArtifact (:509-511); equal at f and -f
// with s the fftshift-ed index.  Two of the three axes are constant along a pass-B column, so a
// butterfly computes them once and each coefficient only adds its H part.
struct AxisGeo {
  int k, nk, dsq, ef, en, odd;
};
TB_HD AxisGeo axis_geo(int k, int n) {
  AxisGeo g;
  g.k = k;
  g.nk = negk(k, n);
  const int s = shifted(k, n), ns = shifted(g.nk, n);
  const int d = s - n / 2, e = 2 * s - (n - 1), en = 2 * ns - (n - 1);
  g.dsq = d * d;
  g.ef = e * e;
  g.en = en * en;
  g.odd = s & 1;
  return g;
}
struct FreqCol {  // W and D parts of a coefficient's geometry
  int kw, kd, nkw, nkd, dsq, ef, en, odd;
};
TB_HD FreqCol freq_col(int kw, int kd, int W, int D) {
  const AxisGeo w = axis_geo(kw, W), d = axis_geo(kd, D);
  return FreqCol{kw, kd, w.nk, d.nk, w.dsq + d.dsq, w.ef + d.ef, w.en + d.en, w.odd + d.odd};
}

// GibbsNoiseLayer mask (stylization_layers.py:99-109): float32 geometry, centre (n-1)/2,
// norm_dist = dist / (alpha * max dist); mask = !(norm_dist > 1)  (NaN -> 1, inf -> 0).
// d2 = e2/4 is an exact quarter-integer, so its float32 sum order is immaterial.
TB_HD bool layer_in(const tb_op& op, int e2) {
  // alpha * max_dist: from the launch arguments, or (op.l != 0) from the layer's device-resident
  // alpha buffer times max_dist in f[1] -- no host round trip for the alpha of Gibbs_GD updates
  const float an = op.l ? (*reinterpret_cast<const float*>(op.l)) * op.f[1] : op.f[0];
  const float nd = f32_div(f32_sqrt((float)e2 * 0.25f), an);
  return !(nd > 1.f);
}

// The target value of a spike: |k| := amp (= exp(intensity)), phase kept
// (filters_and_operators.py:383-390, 927-942) or overridden (parity hook).
TB_HD cf spike_target(const tb_op& op, cf kf) {
  float ph = op.f[1];
  if (ph != ph) {  // NaN -> keep the coefficient's own phase (angle(0) = 0)
    const float m2 = kf.x * kf.x + kf.y * kf.y;
    if (m2 > 0.f) {
      const float inv = 1.f / f32_sqrt(m2);
      return mk(op.f[0] * kf.x * inv, op.f[0] * kf.y * inv);
    }
    return mk(op.f[0], 0.f);
  }
  return mk(op.f[0] * op.f[2], op.f[0] * op.f[3]);  // host passes cos/sin of the override
}

// RandZF draw of one unshifted coefficient: kept iff u > p (utils2.py:70-72 zeroes u <= p)
TB_HD uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
TB_HD float zf_keep(const tb_op& op, uint64_t idx) {
  const float u = (float)(splitmix64(idx ^ (uint64_t)op.l) >> 40) * (1.0f / 16777216.0f);
  return u > op.f[0] ? 1.f : 0.f;
}

// Apply a sample's op program to one stored half-spectrum coefficient.
// Every op is followed by the reference's `.real` (G4: Hermitian symmetrisation);
// on a half spectrum that is exact for symmetric masks, needs (M(f)+M(-f))/2 for
// the off-centre Gibbs masks, and splits a spike into +Delta/2 at f and
// +conj(Delta)/2 at -f.  Consecutive SPIKE ops flagged `reserved = 1` belong to one
// KSpaceSpikeNoise call: they are all measured against the spectrum BEFORE the group
// (the reference writes every location into one log-amplitude array, :936-942).
template <class SO>
TB_HD cf apply_ops(const SO& so, int chan, cf v, const FreqCol& fc, int kh, int H) {
  const AxisGeo h = axis_geo(kh, H);
  cf gbase = v;
  bool in_group = false;
  for (int o = 0; o < so.n; ++o) {   // op fields come straight from the kernarg segment (scalar loads)
    const tb_op& op = so.op[o];
    if (op.kind == TB_OP_SPIKE) {
      if (!in_group || op.reserved != 1) gbase = v;
      in_group = true;
    } else {
      in_group = false;
    }
    if (op.chan >= 0 && op.chan != chan) continue;
    switch (op.kind) {
      case TB_OP_DISK: {
        const int sq = h.dsq + fc.dsq;
        bool in = op.i[0] ? ((int64_t)sq < op.l) : ((float)sq < op.f[0]);
        if (op.i[1]) in = !in;                            // inside_off
        v = in ? v : mk(0.f, 0.f);
      } break;
      case TB_OP_GIBBS: {
        const float m = 0.5f * (((int64_t)(h.ef + fc.ef) <= op.l ? 1.f : 0.f) +
                                ((int64_t)(h.en + fc.en) <= op.l ? 1.f : 0.f));
        v = scl(v, m);
      } break;
      case TB_OP_LAYER: {
        const float m = 0.5f * ((layer_in(op, h.ef + fc.ef) ? 1.f : 0.f) + (layer_in(op, h.en + fc.en) ? 1.f : 0.f));
        v = scl(v, m);
      } break;
      case TB_OP_WRAP: {
        const int nodd = h.odd + fc.odd;
        const float a = op.f[0];
        const float m = nodd == 0 ? 1.f : (nodd == 1 ? a : (nodd == 2 ? a * a : a * a * a));
        v = scl(v, m);
      } break;
      case TB_OP_SPIKE: {
        if (kh == op.i[0] && fc.kw == op.i[1] && fc.kd == op.i[2]) {        // this coefficient is f
          const cf d = sub(spike_target(op, gbase), gbase);
          v = add(v, scl(d, 0.5f));
        }
        if (h.nk == op.i[0] && fc.nkw == op.i[1] && fc.nkd == op.i[2]) {    // this coefficient is -f
          const cf kf = conj(gbase);
          const cf d = sub(spike_target(op, kf), kf);
          v = add(v, scl(conj(d), 0.5f));
        }
      } break;
      case TB_OP_ZF: {  // independent draws at f and -f: the .real symmetrises them
        const uint64_t Wz = (uint64_t)op.i[1], Dz = (uint64_t)op.i[2], ch = (uint64_t)chan * (uint64_t)H;
        const float m = 0.5f * (zf_keep(op, ((ch + (uint64_t)kh) * Wz + (uint64_t)fc.kw) * Dz + (uint64_t)fc.kd) +
                                zf_keep(op, ((ch + (uint64_t)h.nk) * Wz + (uint64_t)fc.nkw) * Dz + (uint64_t)fc.nkd));
        v = scl(v, m);
      } break;
      default: break;
    }
  }
  return v;
}

// ---------------------------------------------------------- pass geometry
// LDS carve of the slab passes (A forward, C inverse), in cf units:
//   [0, NP*PR)          pair rows: z = x[2p] + i x[2p+1], D slots each
//   C0 [W], CN [W]      the real-valued kd=0 / kd=D/2 columns
//   twW [W], twD [D]    twiddle tables
//   posA, posB [Dh]     int: digit-reversed slots of k and D-k
struct SlabGeo {
  int NP, PR, off_c0, off_cn, off_tww, off_twd, off_pos, total_cf;
};

TB_HD SlabGeo slab_geo(int W, int D) {
  SlabGeo g;
  g.NP = (W + 1) / 2;
  g.PR = D;
  g.off_c0 = g.NP * g.PR;
  g.off_cn = g.off_c0 + W;
  g.off_tww = g.off_cn + ((D % 2 == 0) ? W : 0);
  g.off_twd = g.off_tww + W;
  g.off_pos = g.off_twd + D;
  const int Dh = D / 2 + 1;
  g.total_cf = g.off_pos + (2 * Dh + 1) / 2 + 1;  // ints packed two per cf
  return g;
}

// pass B carve: tile [H][T] + twH[H] + irevH[H] (ints)
struct TileGeo {
  int T, off_tw, off_irev, total_cf;
};
TB_HD TileGeo tile_geo(int H, int T) {
  TileGeo g;
  g.T = T;
  g.off_tw = H * T;
  g.off_irev = g.off_tw + H;
  g.total_cf = g.off_irev + (H + 1) / 2 + 1;
  return g;
}

// column addressing of the W-axis FFT inside the slab: element w of column kd
struct ColAddr {
  const int* posA;
  const int* posB;
  int PR, off_c0, off_cn, Dn, D;  // Dn = D/2 if D even else -1
  struct Pen {
    int e, d, pitch;  // even-row slot, odd-minus-even offset (arithmetic, not a select: hipcc
                      // otherwise turns `w&1 ? o : e` into a dynamically indexed stack array)
    TB_HD int operator()(int w) const { return (w >> 1) * pitch + e + (w & 1) * d; }
  };
  TB_HD Pen pen(int kd) const {
    if (kd == 0) return Pen{off_c0, 1, 2};
    if (kd == Dn) return Pen{off_cn, 1, 2};
    const int a = posA[kd];
    return Pen{a, posB[kd] - a, PR};
  }
  TB_HD int operator()(int kd, int w) const { return pen(kd)(w); }
};

// real pair rows of the slab as the source of the first D stage: z = x[2p] + i x[2p+1]
struct PairSrc {
  const float* xb;
  int64_t sw;
  int W;
  struct Pen {
    const float* r0;
    const float* r1;
    bool has1;
    TB_HD cf ld(int i) const { return mk(r0[i], has1 ? r1[i] : 0.f); }
    TB_HD void st(int, cf) const {}
  };
  TB_HD Pen pen(int p) const {
    const float* r0 = xb + (int64_t)(2 * p) * sw;
    return Pen{r0, r0 + sw, 2 * p + 1 < W};
  }
};

// pair rows of the output as the sink of the last inverse D stage: scale, split re/im into
// rows 2p / 2p+1, track the running min/max (salt-and-pepper MIN/MAX epilogue)
struct PairDst {
  float* yb;
  int64_t sw;
  int W;
  float scale;
  float* lo;
  float* hi;
  struct Pen {
    float* r0;
    float* r1;
    bool has1;
    float scale;
    float* lo;
    float* hi;
    TB_HD cf ld(int) const { return mk(0.f, 0.f); }
    TB_HD void st(int i, cf v) const {
      const float a = v.x * scale;
      r0[i] = a;
      *lo = a < *lo ? a : *lo;
      *hi = a > *hi ? a : *hi;
      if (has1) {
        const float b = v.y * scale;
        r1[i] = b;
        *lo = b < *lo ? b : *lo;
        *hi = b > *hi ? b : *hi;
      }
    }
  };
  TB_HD Pen pen(int p) const {
    float* r0 = yb + (int64_t)(2 * p) * sw;
    return Pen{r0, r0 + sw, 2 * p + 1 < W, scale, lo, hi};
  }
};

template <class Ctx>
TB_HD void slab_tables(Ctx& ctx, cf* lds, const tb_plan_dev& pl, const SlabGeo& g) {
  const int W = pl.W, D = pl.D, Dh = D / 2 + 1;
  cf* tww = lds + g.off_tww;
  cf* twd = lds + g.off_twd;
  int* posA = reinterpret_cast<int*>(lds + g.off_pos);
  int* posB = posA + Dh;
  for (int i = ctx.tid; i < W; i += ctx.nthreads) tww[i] = pl.tw[1][i];
  for (int i = ctx.tid; i < D; i += ctx.nthreads) twd[i] = pl.tw[2][i];
  for (int i = ctx.tid; i < Dh; i += ctx.nthreads) {
    posA[i] = pl.rev_d[i];
    posB[i] = pl.rev_d[i == 0 ? 0 : D - i];
  }
  ctx.sync();
}

// --------------------------------------------------------------- pass A
// forward: real slab x[bc][h][:][:] -> half spectrum S[bc][h][w'][kd]
//   D stage 0 reads HBM into registers, D stages 1.. in LDS, pair unpack in LDS,
//   W stages 0..S-2 in LDS, the last W stage writes HBM from registers.
template <class Ctx, int RS>
TB_HD void pass_a_body(Ctx& ctx, cf* lds, const tb_plan_dev& pl, const float* __restrict__ x, int64_t sx_bc,
                       int64_t sx_h, int64_t sx_w, cf* __restrict__ S, int bc, int h) {
  const int W = pl.W, D = pl.D, Dh = D / 2 + 1;
  const SlabGeo g = slab_geo(W, D);
  slab_tables(ctx, lds, pl, g);
  const cf* tww = lds + g.off_tww;
  const cf* twd = lds + g.off_twd;
  const int* posA = reinterpret_cast<const int*>(lds + g.off_pos);
  const int* posB = posA + Dh;
  const float* xb = x + bc * sx_bc + h * sx_h;
  const tb_axis& axd = pl.ax[2];
  const tb_axis& axw = pl.ax[1];
  const auto rows = lds_acc(lds, RowAddr{g.PR});
  const FastDiv fDh = FastDiv::make(Dh);
  if (axd.nst == 0) {
    const FastDiv fD = FastDiv::make(D);
    copy_batched<kCopyUnroll>(
        ctx, g.NP * D, [&](int t) { return PairSrc{xb, sx_w, W}.pen(fD.div(t)).ld(t - fD.div(t) * D); },
        [&](int t, cf v) { lds[fD.div(t) * g.PR + (t - fD.div(t) * D)] = v; });
    ctx.sync();
  } else {
    stage<Ctx, true, RS>(ctx, PairSrc{xb, sx_w, W}, rows, twd, axd.radix[0], D, 1, g.NP, D, false);
    ctx.sync();
    dif_stages<Ctx, RS>(ctx, rows, twd, axd, 1, axd.nst, g.NP, false);
  }
  // unpack the pair spectra in place (each unit owns the two slots it reads)
  const int Dn = (D % 2 == 0) ? D / 2 : -1;
  const int nun = g.NP * Dh;
  for (int t = ctx.tid; t < nun; t += ctx.nthreads) {
    const int p = fDh.div(t), k = t - p * Dh;
    cf* row = lds + p * g.PR;
    const int w0 = 2 * p;
    if (k == 0 || k == Dn) {
      const cf z = row[posA[k]];
      cf* col = lds + (k == 0 ? g.off_c0 : g.off_cn);
      col[w0] = mk(z.x, 0.f);
      if (w0 + 1 < W) col[w0 + 1] = mk(z.y, 0.f);
    } else {
      const cf zk = row[posA[k]], zm = conj(row[posB[k]]);
      const cf xa = scl(add(zk, zm), 0.5f);
      const cf dd = scl(sub(zk, zm), 0.5f);
      row[posA[k]] = xa;
      row[posB[k]] = mk(dd.y, -dd.x);  // (zk - zm) / (2i)
    }
  }
  ctx.sync();
  const ColAddr ca{posA, posB, g.PR, g.off_c0, g.off_cn, Dn, D};
  const auto cols = lds_acc(lds, ca);
  cf* Sb = S + ((int64_t)bc * pl.H + h) * (int64_t)W * Dh;
  if (axw.nst == 0) {
    copy_batched<kCopyUnroll>(
        ctx, W * Dh, [&](int t) { const int w = fDh.div(t); return lds[ca(t - w * Dh, w)]; },
        [&](int t, cf v) { Sb[t] = v; });
  } else {
    dif_stages<Ctx, RS>(ctx, cols, tww, axw, 0, axw.nst - 1, Dh, true);
    const int sl = axw.nst - 1, P = prefix_product(axw, sl);
    stage<Ctx, true, RS>(ctx, cols, StridedAcc{Sb, 1, Dh}, tww, axw.radix[sl], W / P, P, Dh, W, true);
  }
}

// --------------------------------------------------------------- pass B
// per (bc, tile of T spectrum columns): H stage 0 from HBM, H stages in LDS, the last forward
// stage fused with the op program and the first inverse stage in registers, inverse stage 0
// back to HBM.
// the op program of one pass-B tile column: per-column geometry once, per-coefficient H part
template <class SO>
struct KOps {
  const SO& so;
  int chan, j0, Dh;
  FastDiv fDh;
  const int* irev;    // H slot -> frequency (LDS)
  const int* irev_w;  // W slot -> frequency
  int H, W, D;
  TB_HD FreqCol col(int c) const {
    const int j = j0 + c;
    const int wp = fDh.div(j);
    return freq_col(irev_w[wp], j - wp * Dh, W, D);
  }
  TB_HD cf operator()(const FreqCol& fc, int pos, cf v) const { return apply_ops(so, chan, v, fc, irev[pos], H); }
};

template <class Ctx, int RS, class SO>
TB_HD void pass_b_body(Ctx& ctx, cf* lds, const tb_plan_dev& pl, cf* __restrict__ S, int bc, int tile, int T,
                       const SO& so, int chan) {
  const int H = pl.H, W = pl.W, D = pl.D, Dh = D / 2 + 1;
  const int ncols_all = W * Dh;
  const int j0 = tile * T;
  const int nc = (ncols_all - j0) < T ? (ncols_all - j0) : T;
  const TileGeo g = tile_geo(H, T);
  cf* tw = lds + g.off_tw;
  int* irev = reinterpret_cast<int*>(lds + g.off_irev);
  for (int i = ctx.tid; i < H; i += ctx.nthreads) { tw[i] = pl.tw[0][i]; irev[i] = pl.irev_h[i]; }
  ctx.sync();
  cf* Sb = S + (int64_t)bc * H * ncols_all + j0;
  const StridedAcc gacc{Sb, 1, ncols_all};
  const KOps<SO> ops{so, chan, j0, Dh, FastDiv::make(Dh), irev, pl.irev_w, H, W, D};
  const tb_axis& ax = pl.ax[0];
  if (ax.nst == 0) {  // H == 1: the op program alone
    for (int t = ctx.tid; t < nc; t += ctx.nthreads) Sb[t] = ops(ops.col(t), 0, Sb[t]);
    return;
  }
  if (ax.nst == 1) {  // one radix: HBM -> DFT -> ops -> IDFT -> HBM, no LDS round trip
    stage_mid<Ctx, RS>(ctx, gacc, gacc, ax.radix[0], nc, H, ops, true);
    return;
  }
  const auto la = lds_acc(lds, TileAddr{T});
  stage<Ctx, true, RS>(ctx, gacc, la, tw, ax.radix[0], H, 1, nc, H, true);
  ctx.sync();
  dif_stages<Ctx, RS>(ctx, la, tw, ax, 1, ax.nst - 1, nc, true);
  stage_mid<Ctx, RS>(ctx, la, la, ax.radix[ax.nst - 1], nc, H, ops, true);
  ctx.sync();
  dit_stages<Ctx, RS>(ctx, la, tw, ax, 1, ax.nst - 1, nc, true);
  stage<Ctx, false, RS>(ctx, la, gacc, tw, ax.radix[0], H, 1, nc, H, true);
}

// --------------------------------------------------------------- pass C
// inverse: S[bc][h] -> y[bc][h][:][:] (scaled 1/N), pad columns [D, D+ypad) zeroed,
// running (min, max) of the written values for salt-and-pepper.
template <class Ctx, int RS>
TB_HD void pass_c_body(Ctx& ctx, cf* lds, const tb_plan_dev& pl, const cf* __restrict__ S, float* __restrict__ y,
                       int64_t sy_bc, int64_t sy_h, int64_t sy_w, int ldy_pad, int bc, int h, float scale,
                       float* vmin, float* vmax) {
  const int W = pl.W, D = pl.D, Dh = D / 2 + 1;
  const SlabGeo g = slab_geo(W, D);
  slab_tables(ctx, lds, pl, g);
  const cf* tww = lds + g.off_tww;
  const cf* twd = lds + g.off_twd;
  const int* posA = reinterpret_cast<const int*>(lds + g.off_pos);
  const int* posB = posA + Dh;
  const int Dn = (D % 2 == 0) ? D / 2 : -1;
  const ColAddr ca{posA, posB, g.PR, g.off_c0, g.off_cn, Dn, D};
  const auto cols = lds_acc(lds, ca);
  const auto rows = lds_acc(lds, RowAddr{g.PR});
  cf* Sb = const_cast<cf*>(S) + ((int64_t)bc * pl.H + h) * (int64_t)W * Dh;
  const tb_axis& axd = pl.ax[2];
  const tb_axis& axw = pl.ax[1];
  const FastDiv fDh = FastDiv::make(Dh);
  if (axw.nst == 0) {
    copy_batched<kCopyUnroll>(
        ctx, W * Dh, [&](int t) { return Sb[t]; },
        [&](int t, cf v) { const int w = fDh.div(t); lds[ca(t - w * Dh, w)] = v; });
    ctx.sync();
  } else {
    const int sl = axw.nst - 1, P = prefix_product(axw, sl);
    stage<Ctx, false, RS>(ctx, StridedAcc{Sb, 1, Dh}, cols, tww, axw.radix[sl], W / P, P, Dh, W, true);
    ctx.sync();
    dit_stages<Ctx, RS>(ctx, cols, tww, axw, 0, axw.nst - 1, Dh, true);
  }
  // repack rows (2p, 2p+1) into the pair spectrum z = X_a + i X_b (digit-reversed slots)
  const int nun = g.NP * Dh;
  for (int t = ctx.tid; t < nun; t += ctx.nthreads) {
    const int p = fDh.div(t), k = t - p * Dh;
    cf* row = lds + p * g.PR;
    const int w0 = 2 * p;
    const bool has_b = (w0 + 1 < W);
    if (k == 0 || k == Dn) {
      const cf* col = lds + (k == 0 ? g.off_c0 : g.off_cn);
      row[posA[k]] = mk(col[w0].x, has_b ? col[w0 + 1].x : 0.f);   // c2r keeps Re of DC/Nyquist
    } else {
      const cf xa = row[posA[k]];
      const cf xb = has_b ? row[posB[k]] : mk(0.f, 0.f);
      row[posA[k]] = mk(xa.x - xb.y, xa.y + xb.x);         // xa + i xb
      row[posB[k]] = mk(xa.x + xb.y, -xa.y + xb.x);        // conj(xa) + i conj(xb)
    }
  }
  ctx.sync();
  float* yb = y + bc * sy_bc + h * sy_h;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  if (axd.nst == 0) {
    for (int t = ctx.tid; t < W; t += ctx.nthreads) {
      const cf z = lds[(t >> 1) * g.PR];
      const float v = ((t & 1) ? z.y : z.x) * scale;
      yb[t * sy_w] = v;
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
  } else {
    dit_stages<Ctx, RS>(ctx, rows, twd, axd, 1, axd.nst, g.NP, false);
    stage<Ctx, false, RS>(ctx, rows, PairDst{yb, sy_w, W, scale, &lo, &hi}, twd, axd.radix[0], D, 1, g.NP, D,
                          false);
  }
  if (ldy_pad > 0) {
    const FastDiv fp = FastDiv::make(ldy_pad);
    for (int t = ctx.tid; t < W * ldy_pad; t += ctx.nthreads) {
      const int w = fp.div(t);
      yb[w * sy_w + D + (t - w * ldy_pad)] = 0.f;
    }
  }
  *vmin = lo;
  *vmax = hi;
}

}  // namespace tb
