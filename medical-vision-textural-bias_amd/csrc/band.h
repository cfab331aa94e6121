// band.h -- band-limited ("pruned") k-space filter passes.
//
// The reference's drivers start their chains with a small low-pass: RandFourierDiskMaskd(r=12.5)
// keeps 8,217 of the 8.9 M coefficients of a 240x240x155 volume
// (10_scripts/127_.../..._3modalities.py:171-174, source_code/filters_and_operators.py:236-252).
// Everything after it in k-space is diagonal (wrap, further masks, filters_and_operators.py:503-515)
// or a point update (plane-wave / k-space spikes, :383-390, :936-942).  So the whole program's
// output spectrum lives in a small box around DC plus a handful of spike points, and the full
// mixed-radix FFT round trip (passes A/B/C, 32 B/voxel of HBM traffic) is replaced by:
//
//   A' k_band_fwd   per 16-row strip of a (bc, h) slab, each wave streaming its own contiguous,
//                   balanced range of strips (next strip prefetched into registers, staged in the
//                   wave's own LDS region, no workgroup barriers): pruned real DFT along D (kd in
//                   [0, NDk), d-symmetric, MFMA) then pruned DFT along W (kw in [-KW, KW]) accumulated
//                   in registers; a slab shared by several waves gets one partial sum per wave
//                   (P[bc][h][seg][NW][NDk], seg < BAND_FWD_SEGS) that pass B' adds.  Reads the image once.
//   B' k_band_mid   per (bc, kh, 64 columns): pruned DFT along H (kh and -kh at once), the
//                   sample's op program (apply_ops, the same code as pass B) on every box
//                   coefficient, stored as the kh/-kh sum and difference AB[bc][kh][col]; the
//                   out-of-box spike points' coefficients = the program applied to 0.
//   C' k_band_inv   per (bc, h) slab: inverse H and W on the box (VALU), then the C2R along D as
//                   an f32 MFMA product [rows x 2(NDk+points)] . [2(NDk+points) x D+pad] whose
//                   second factor is the cos/sin table with zero pad columns -- so the U-Net's
//                   D-padding comes out of the MFMA as zeros -- stored straight from the
//                   accumulators; per-sample min/max epilogue.  Writes the image once.
//
// Exactness: the box contains every coefficient the low-pass keeps (host-checked with the
// mask's own arithmetic), a spike outside the box lands on a coefficient that is zero after the
// low-pass, so its final value is the program applied to 0 (SURVEY G4/G5 and DESIGN.md).
#pragma once

#include "kernels.h"

namespace tb {

constexpr int BAND_NT = 256;
constexpr int BAND_MAX_PTS = 8;    // out-of-box half-spectrum spike points per sample
constexpr int BAND_ROWS_A = 64;    // image rows per pass-A' chunk (one per lane)
constexpr int BAND_MAX_NDK = 32;
constexpr int BAND_MAX_KH = 31;    // box half-height
constexpr int BAND_MAX_ZCOL = 1536; // box columns (kw, kd) per slab in pass B2''s LDS (r = 25.1 at 240^2 x 155: 1,326)

struct BandPt {
  int16_t kh, kw, kd, pad;  // unsigned frequency of the stored (kd <= D/2) coefficient
};
struct BandSamplePts {
  int n;
  BandPt p[BAND_MAX_PTS];
};

struct BandGeo {
  int KH, KW, NDk;  // box: signed kh in [-KH, KH], signed kw in [-KW, KW], kd in [0, NDk)
  int NW, ncol;     // 2 KW + 1, NW * NDk  (a "column" = one (kw, kd) pair of the box)
  int KS;           // k-steps of the inverse D MFMA: NDk band columns + the launch's max points
  int NCOL;         // folded output columns of the MFMA n-tiles: 32 * ceil((D/2 + 1) / 32)
  int cat;          // 1: split-f16 pass C' (k_band_inv16) -- every sample's points get their own V rows
  int PT;           // cat: points of the whole launch (rows 2 (NDk + p0[s] + j) hold sample s's point j)
  int NTD;          // cat: 32-column tiles of a stored output row, ceil((D + pad) / 32)
};
// rows of V (2 per kd band column / point) and its 32-row MFMA tiles
TB_HD int band_rows(const BandGeo& g) { return 2 * (g.cat ? g.NDk + g.PT : g.KS); }

// Pass A''s division of the launch's T = slabs x nst 16-row strips among G waves: wave w takes
// strips [w T / G, (w + 1) T / G).  G <= T / ceil(nst / 2), so a slab spans at most 3 waves.
// (T + 1) G < 2^32 (host-checked): 32-bit arithmetic.
constexpr int BAND_FWD_SEGS = 3;
// Longest D a band plan takes (the passes stage D-long rows in LDS well below this); plans past it
// build no band tables (tds, tbt: O(D^2) entries).
constexpr int BAND_MAX_D = 4096;
constexpr int BAND_FWD_ROWS = 16;  // rows per strip (one per lane of a 16x16x4 MFMA row)
struct FwdSplit {
  uint32_t T, G, nst;
};
TB_HD uint32_t fwd_start(const FwdSplit& s, uint32_t w) { return w * s.T / s.G; }
TB_HD uint32_t fwd_wave_of(const FwdSplit& s, uint32_t t) { return ((t + 1) * s.G - 1) / s.T; }
// partial sums of a slab = waves that hold one of its strips
TB_HD int fwd_nseg(const FwdSplit& s, uint32_t slab) {
  return (int)(fwd_wave_of(s, slab * s.nst + s.nst - 1) - fwd_wave_of(s, slab * s.nst)) + 1;
}

struct BandFwdArgs {
  tb_plan_dev pl;
  const float* x;
  int64_t sbc, sh, sw;
  cf* P;            // [bc][H][BAND_FWD_SEGS][ncol] partial sums (bc absolute)
  int bc0, nbc;
  BandGeo g;
  int diag;         // measurement only (TEXBIAS_BAND_DIAG): skip stages, results invalid
  const float* tbt; // [2][KSd][2][64] B fragments of the folded D product (plan table)
  FwdSplit split;   // set by launch_band_fwd
  int vec;          // contiguous 16-B aligned rows (sw == D, 16-B aligned base and slab strides)
  const void* tbt16;  // compiled D: [KS16][cos/sin][hi/lo][64][8 halves] split-f16 D-product B fragments
};
// Pass A' D product in split f16 (compiled D): 32-wide k-steps of the folded d in [0, D/2]
TB_HD constexpr int band_fwd16_ks(int D) { return (D / 2 + 1 + 31) / 32; }
constexpr float BAND_FWD16_TSCALE = 256.f;  // the table is stored x 2^8 (no f16 subnormals)

struct BandMidArgs {
  tb_plan_dev pl;
  cf* P;            // pass A' partial sums; pass B' writes Z over each slab's first slot
  float4* AB;       // [bc][KH + 1][ncol]: (Q'(kh) + Q'(-kh), Q'(kh) - Q'(-kh))
  cf* pts;          // [bc][BAND_MAX_PTS]
  float* M2F;       // [bc][H][VT][KV][64]: pass C''s V-product A fragments (written by B2')
  float scale;      // 1 / (H W D)
  int bc0, C, cofs, nbc;
  BandGeo g;
  FwdSplit split;   // pass A''s strip division (how many partial sums each slab has)
  BandSamplePts sp[TB_MAX_BATCH];
  int p0[TB_MAX_BATCH];  // g.cat: the first V point row (pair) of each sample of the launch
  int16_t pkd[TB_MAX_BATCH * BAND_MAX_PTS];  // g.cat: kd of the launch's points in row order
  void* T16;        // g.cat: synthesis-table fragments for pass C' (written by k_band_tab16)
  uint32_t* mm;     // g.cat: per-sample min/max keys, initialised here for pass C''s atomics (or null)
  const float* tds; // g.cat: [D/2 + 1][2][NCOL] folded synthesis table (plan table)
  BatchOps ops;
  uint32_t* cnt;    // pass C''s arrival counter, zeroed here (B' runs before every C')
};

struct BandInvArgs {
  tb_plan_dev pl;
  const float* M2F; // [bc][H][VT][KV][64] V-product A fragments (pass B2')
  const float4* AB;
  const cf* pts;
  float* y;
  int64_t sbc, sh, sw;
  int ypad, bc0, C, cofs, nbc;
  float scale;      // 1 / (H W D)
  uint32_t* mm;     // per-sample min/max keys (written, not accumulated: whole samples per launch)
  float2* mmp;      // [b][C H ntw] per-(slab, 32-row tile) (min, max) partials
  BandGeo g;
  BandSamplePts sp[TB_MAX_BATCH];
  int diag;
  const float* tds; // [D/2 + 1][2][NCOL] folded synthesis table (plan table)
  const void* T16;  // g.cat: split-f16 synthesis-table fragments (k_band_tab16)
  uint32_t* cnt;    // g.cat: arrival counter (zeroed by pass B'); the last workgroup writes the keys
  int slots;        // g.cat: slab slots per fragment batch (set by launch_band_inv)
};

// Pass A': LDS row pitch of a staged strip.  Odd D: D (the strip is one contiguous run, 16-B
// vectors land aligned); compiled D with D % 4 == 0: D + 4 (16-B rows, conflict-free folded reads);
// otherwise D + 1 (element-wise staging).
TB_HD int band_fwd_pitch(int D, bool ct) { return (D & 1) ? D : (ct && (D & 3) == 0) ? D + 4 : D + 1; }
// compiled pass-A' kernels (D known at compile time, D-product table in registers)
TB_HD bool band_fwd_ct(int D, int NT2) { return NT2 == 1 && (D == 155 || D == 128); }
// floats of one wave's region: the staged strip (+8 slack) or, at a segment end, its O partials
// [cos/sin][re/im][KWT][NT2][64 lanes][4] -- whichever is larger
TB_HD int band_fwd_xw(int P, int NT2, int KWT) {
  const int xn = BAND_FWD_ROWS * P + 8, ob = 2 * 2 * KWT * NT2 * 64 * 4;
  return xn > ob ? xn : ob;
}
// LDS bytes of pass A': [W twiddles][D-product table (runtime D only)][4 wave regions]
TB_HD size_t band_lds_fwd(const BandGeo& g, int W, int D, bool ct) {
  const int NT2 = g.NDk <= 16 ? 1 : 2, KWT = g.KW < 16 ? 1 : 2, KSd = (D / 2 + 1 + 3) / 4;
  const size_t tw = ((size_t)W * 8 + 15) & ~(size_t)15;
  const size_t bt = ct ? 0 : (size_t)NT2 * KSd * 128 * 4;
  return tw + bt + (size_t)4 * band_fwd_xw(band_fwd_pitch(D, ct), NT2, KWT) * 4;
}
#ifndef TB_BAND_SLOTS
#define TB_BAND_SLOTS 3
#endif
constexpr int BAND_SLOTS = TB_BAND_SLOTS;  // slabs whose pass-C' inputs a workgroup holds in LDS at once
constexpr int BAND_STG_P = 36;  // pitch (floats) of a wave's staged 32 x 32 output half-tile
struct BandInvCarve {  // byte offsets of the pass-C' LDS regions (16-B aligned)
  int bimg, tww, frag, prow, pkw, stg, total;
};
TB_HD int band_al16(int b) { return (b + 15) & ~15; }
TB_HD int band_vt(const BandGeo& g) { return band_rows(g) <= 32 ? 1 : 2; }  // 32-row tiles of V
TB_HD int band_kv(const BandGeo& g) { return g.KW + 1 + (g.KS - g.NDk); }
TB_HD BandInvCarve band_inv_carve(const BandGeo& g, int W, int D) {
  (void)D;
  const int npm = g.KS - g.NDk;
  BandInvCarve c;
  c.bimg = 0;                                         // [2 NDk][NCOL] band rows of the synthesis table
  c.tww = band_al16(c.bimg + 2 * g.NDk * g.NCOL * 4); // [W] twiddles
  c.frag = band_al16(c.tww + W * 8);                  // [SLOTS][VT KV 64] V-product fragments
  c.prow = band_al16(c.frag + BAND_SLOTS * band_vt(g) * band_kv(g) * 64 * 4);  // [SLOTS][2 npm + 4][NCOL]
  c.pkw = band_al16(c.prow + BAND_SLOTS * (2 * npm + 4) * g.NCOL * 4);  // [SLOTS][BAND_MAX_PTS] point kw
  c.stg = band_al16(c.pkw + BAND_SLOTS * BAND_MAX_PTS * 4);  // [4 waves][32][BAND_STG_P] staging
  c.total = band_al16(c.stg + 4 * 32 * BAND_STG_P * 4);
  return c;
}

// Split-f16 pass C' (k_band_inv16): the unfolded synthesis table as MFMA B fragments
// [NTD][nch][hi/lo][64 lanes][8 halves] (NTD 32-column tiles of the stored row, nch 16-row chunks
// of V), then the W twiddles, BAND_SLOTS16 slabs' V-product fragments, the slabs' point kw.
#ifndef TB_BAND_SLOTS16
#define TB_BAND_SLOTS16 3
#endif
constexpr int BAND_SLOTS16 = TB_BAND_SLOTS16;
// slab slots of a workgroup of nw waves (16 waves: one workgroup per CU takes ~4x the units)
TB_HD constexpr int band_slots16(int nw) { return nw <= 4 ? BAND_SLOTS16 : 12; }
TB_HD int band_nch(const BandGeo& g) { return (band_rows(g) + 15) / 16; }
TB_HD int band_t16_bytes(const BandGeo& g) { return g.NTD * band_nch(g) * 2 * 64 * 16; }
struct BandInv16Carve {
  int tab, tww, frag, pkw, total;
};
TB_HD BandInv16Carve band_inv16_carve(const BandGeo& g, int W, int slots = BAND_SLOTS16) {
  BandInv16Carve c;
  c.tab = 0;
  c.tww = band_al16(band_t16_bytes(g));
  c.frag = band_al16(c.tww + W * 8);
  c.pkw = band_al16(c.frag + slots * band_vt(g) * band_kv(g) * 64 * 4);
  c.total = band_al16(c.pkw + slots * BAND_MAX_PTS * 4);
  return c;
}

// Pass B' (k_band_hcol): 16 box columns per workgroup; LDS = their partial sums for every slab (+1
// zero row), the H twiddles, the [C; S] product tiles, the G rows of the inverse.
#ifndef TB_HC_NW
#define TB_HC_NW 8  // waves per pass-B' workgroup (they split h): the launch is only ncol / 16 x nbc
                    // workgroups (168 at C3), so its latency wants the waves (4: 33.7 us with B2', 8: 30.8)
#endif
constexpr int BAND_HC_NW = TB_HC_NW;
TB_HD size_t band_hc_lds(int H, int KH) {
  const int mt = KH + 1 <= 16 ? 1 : 2;
  return (size_t)(H + 1) * 16 * 8 + (size_t)H * 8 + (size_t)mt * 1024 * 4 + (size_t)2 * (KH + 1) * 32 * 4 +
         (size_t)BAND_HC_NW * mt * 1024 * 4;  // + the waves' forward sums
}

// workspace carve (bytes from the workspace base) for `bcn` volume-channels
struct BandWs {
  size_t off_P, off_AB, off_pts, off_mmp, off_m2f, off_t16, off_cnt, total;
};
TB_HD BandWs band_ws(const BandGeo& g, int H, int bcn) {
  BandWs w;
  w.off_P = 0;
  w.off_AB = (size_t)bcn * H * BAND_FWD_SEGS * g.ncol * 8;
  w.off_AB = (w.off_AB + 255) & ~(size_t)255;
  w.off_pts = w.off_AB + (size_t)bcn * (g.KH + 1) * g.ncol * 16;
  w.off_mmp = w.off_pts + (size_t)bcn * BAND_MAX_PTS * 8;
  w.off_m2f = w.off_mmp + (size_t)bcn * H * 32 * 8;  // (min, max) per (slab, 32-row tile), W <= 1024
  w.off_m2f = (w.off_m2f + 255) & ~(size_t)255;
  w.off_t16 = w.off_m2f + (size_t)bcn * H * band_vt(g) * band_kv(g) * 64 * 4;
  w.off_t16 = (w.off_t16 + 255) & ~(size_t)255;
  w.off_cnt = (w.off_t16 + (size_t)band_t16_bytes(g) + 255) & ~(size_t)255;  // pass C' arrival counter
  w.total = w.off_cnt + 256;
  return w;
}

// Launchers (kern_band.hip).  ncu = compute units (persistent slab grids).
hipError_t launch_band_fwd(BandFwdArgs& a, int ncu, hipStream_t st);  // sets a.split
bool band_fwd_use_ct(int D, int NT2);  // the compiled-D pass-A' kernel runs for this D
hipError_t launch_band_mid(const BandMidArgs& a, hipStream_t st);
hipError_t launch_band_inv(BandInvArgs& a, int ncu, hipStream_t st);  // g.cat: k_band_inv16 (sets a.slots)
hipError_t launch_band_minmax(const float2* mmp, uint32_t* mm, int bc0, int C, int nbc, int H, int W, hipStream_t st);

// identity samples (empty program): strided copy + zero D-padding + min/max
struct CopyArgs {
  const float* x;
  int64_t xsbc, xsh, xsw;
  float* y;
  int64_t ysbc, ysh, ysw;
  int H, W, D, ypad, bc0, C, nbc;
  uint32_t* mm;
};
hipError_t launch_copy_pad(const CopyArgs& a, hipStream_t st);

}  // namespace tb
