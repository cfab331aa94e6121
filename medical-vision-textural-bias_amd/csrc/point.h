// point.h -- closed-form route for programs made only of k-space spikes.
//
// RandPlaneWaves_ellipsoid (source_code/filters_and_operators.py:370-393) and KSpaceSpikeNoise
// (:906-983) change single coefficients of the spectrum and take `.real` of the inverse FFT.  For
// spikes at frequencies f_j that do not touch each other (no two equal or conjugate in a shared
// channel) that is, exactly,
//   y = x + Re( sum_j Delta_j exp(2 pi i f_j . n / N) ) / N,   Delta_j = target_j(K(f_j)) - K(f_j),
// with K(f) = sum_n x[n] exp(-2 pi i f . n / N) one coefficient of the forward DFT.
// Three launches instead of a spectrum round trip: the coefficients K_bc(f_j) (reads x once),
// Delta_j / N per (bc, j), and the streaming add (reads x, writes y + padding + min/max keys):
// 12 B per voxel against the full-spectrum route's 32.
#pragma once

#include "kernels.h"

namespace tb {

constexpr int POINT_NT = 256;
constexpr int POINT_WG = 2048;  // most workgroups a launch uses (8 per CU)

struct PointArgs {
  int H, W, D;
  const float* x;
  int64_t xsbc, xsh, xsw;
  float* y;
  int64_t ysbc, ysh, ysw;
  int ypad, bc0, C, nbc;  // bc0 = first sample * C (absolute); ops.s[i] = the run's i-th sample
  int parts;              // workgroups per volume-channel (each a contiguous range of the volume's quads)
  int parts_apply;        // the same for k_point_apply (its own occupancy)
  int namax;              // most spikes any volume-channel of the launch has (twiddle-table stride)
  uint32_t* mm;           // per-sample min/max keys (written by the last apply workgroup) or null
  double* part;           // [nbc][parts][TB_MAX_OPS][2] per-workgroup coefficient sums
  float* delta;           // [nbc][TB_MAX_OPS][2] Delta_j / N (zero for ops that skip the channel)
  float2* mmp;            // [nbc][parts] per-workgroup (min, max) of the output
  uint32_t* cnt;          // arrival counter of the apply workgroups (zeroed by k_point_delta)
  BatchOps ops;
};

// workspace carve for nbc volume-channels
struct PointWs {
  size_t part, delta, mmp, cnt, total;
};
inline PointWs point_ws(int nbc) {
  PointWs w;
  w.part = 0;  // nbc * parts <= POINT_WG + nbc: regions sized for that, so the carve grows with nbc
  w.delta = ((size_t)(POINT_WG + nbc) * TB_MAX_OPS * 16 + 255) & ~(size_t)255;
  w.mmp = (w.delta + (size_t)nbc * TB_MAX_OPS * 8 + 255) & ~(size_t)255;
  w.cnt = (w.mmp + (size_t)(POINT_WG + nbc) * 8 + 255) & ~(size_t)255;
  w.total = w.cnt + 256;
  return w;
}

// Every op is a spike and no two touch (same or conjugate frequency in an overlapping channel).
bool point_program(const tb_sample_ops& s, int H, int W, int D);
// The kernels' index codes and 32-bit row offsets hold: H <= 2048, W <= 1024, (D + pad + 3) / 4 < 1024
// quads, and every row of a volume-channel of x and y within 2^32 elements of its first.
inline bool point_strides_ok(int H, int W, int D, int ypad, const int64_t* xs, const int64_t* ys) {
  if (H > 2048 || W > 1024 || (D + ypad + 3) / 4 >= 1024) return false;
  const int64_t lim = (int64_t)1 << 32;
  return (int64_t)(H - 1) * xs[1] + (int64_t)(W - 1) * xs[2] + D < lim &&
         (int64_t)(H - 1) * ys[1] + (int64_t)(W - 1) * ys[2] + D + ypad < lim && xs[1] >= 0 && xs[2] >= 0 &&
         ys[1] >= 0 && ys[2] >= 0;
}
// Sets a.parts / a.parts_apply: one round of resident workgroups per launch (ncu x occupancy, at most
// POINT_WG), split evenly over the launch's volume-channels.
void point_grid(PointArgs& a, int ncu);
hipError_t launch_point(const PointArgs& a, hipStream_t st, int stage);  // stage 0: K, 1: Delta, 2: apply

}  // namespace tb
