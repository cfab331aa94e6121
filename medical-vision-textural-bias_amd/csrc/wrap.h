// wrap.h -- separable route for programs made only of wrap-around ops.
//
// WrapArtifact (source_code/filters_and_operators.py:503-515) multiplies every shifted-spectrum
// coefficient by alpha once per axis whose shifted index is odd, i.e. by the product of three 1-D
// masks m_a(f) = alpha^[(f + n_a/2) mod n_a odd].  Each m_a is symmetric (m(f) = m(-f)), so the filter is
// a real, separable circulant: y = T_h T_w T_d x, with no spectrum needed:
//   even axis n:  m(f) = (1+alpha)/2 + s (1-alpha)/2 (-1)^f,  s = (-1)^(n/2)
//                 => (T x)[t] = a x[t] + b x[(t + n/2) mod n],  a = (1+alpha)/2, b = s (1-alpha)/2
//   odd axis n:   a dense n-point circulant k[j] = delta_j + (alpha - 1) q[j],
//                 q[j] = (1/n) sum_f [(f + (n-1)/2) mod n odd] cos(2 pi f j / n)   (float64, per plan)
// H and W even (the BraTS 240 x 240): the four rows {h, h+H/2} x {w, w+W/2} of a "quad" map onto
// themselves, so a work unit reads each quad of rows once, combines them with the 2-tap weights and
// applies T_d along the contiguous row:
//   D even:  T_d is 2-tap too -- k_wrap_even, 8 voxels in, 8 out, nothing but FMAs;
//   D odd:   T_d as a matrix product on the f16 matrix cores in split precision (k_wrap_dgemm):
//            Y^T (d_out x rows) = K^T (d_out x d_in) . X^T (d_in x rows), K and X each an f16 hi/lo
//            pair (K scaled by 2^6, X by a per-unit power of two), three products, f32 accumulation;
//            K^T's fragments come from a 10.75 KB LDS table of the circulant (8 shifted copies so
//            every lane's 8 entries are one aligned 16-B read).
// One read and one write of the image: 4 + 4 (+ padding) B per voxel against the full route's 32.
// Per-sample min/max keys (the salt-and-pepper MIN/MAX) from per-workgroup partials, reduced by the
// last workgroup to arrive (store_partial / arrive_last, kernels.h).
#pragma once

#include "kernels.h"

namespace tb {

constexpr int WRAP_NT = 256;       // 4 waves per workgroup
constexpr int WRAP_MAX_WG = 2048;  // most workgroups a launch uses (partials carve)
constexpr int WRAP_MAX_COLS = 256; // D odd: D + pad <= 256 (16 output tiles of 16 columns)

struct WrapArgs {
  int H, W, D;
  const float* x;
  int64_t xsbc, xsh, xsw;
  float* y;
  int64_t ysbc, ysh, ysw;
  int ypad, bc0, C, nbc;  // bc0 = first sample * C (absolute)
  // per sample of the launch: 2-tap weights of the H, W (and, D even, D) axes
  float ah[TB_MAX_BATCH], bh[TB_MAX_BATCH], aw[TB_MAX_BATCH], bw[TB_MAX_BATCH], ad[TB_MAX_BATCH], bd[TB_MAX_BATCH];
  float alpha;            // D odd: the launch's (uniform) D-axis alpha for the circulant table
  const double* q;        // D odd: q[j], j < D (plan table)
  int RS;                 // D odd: floats between the staged role chunks of a unit (>= 4 D, multiple of 4)
  int region;             // D odd: floats of one wave's staging region
  int vec;                // 16-B loads / stores (alignment checked on the host)
  uint32_t* mm;           // per-sample min/max keys, or null
  float2* mmp;            // [gridDim.x][TB_MAX_BATCH] per-workgroup (min, max)
  uint32_t* cnt;          // arrival counter (zeroed before the launch)
};

// workspace carve (partials + counter), bytes
inline size_t wrap_ws_bytes() { return (size_t)WRAP_MAX_WG * TB_MAX_BATCH * 8 + 256; }

// The program is wrap ops only; *alpha = their product (the per-axis masks multiply).
bool wrap_program(const tb_sample_ops& s, float* alpha);
// The shape has a separable route (H, W even; D even, or D odd with D + pad <= WRAP_MAX_COLS).
bool wrap_shape_ok(int H, int W, int D, int ypad);
// q[j] of the odd-D circulant (host, float64), j < D.
void wrap_q_table(int D, double* q);
// Fills a.ah.. from alpha[i] for the launch's samples, the grid, LDS layout; launches.
hipError_t launch_wrap(WrapArgs& a, const float* alpha, int nb, int ncu, hipStream_t st);

}  // namespace tb
