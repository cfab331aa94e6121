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

struct PointArgs {
  int H, W, D;
  const float* x;
  int64_t xsbc, xsh, xsw;
  float* y;
  int64_t ysbc, ysh, ysw;
  int ypad, bc0, C, nbc;  // bc0 = first sample * C (absolute); ops.s[i] = the run's i-th sample
  uint32_t* mm;           // per-sample min/max keys (atomic; reset by the caller) or null
  double* part;           // [nbc][H * parts][TB_MAX_OPS][2] per-workgroup coefficient sums
  float* delta;           // [nbc][TB_MAX_OPS][2] Delta_j / N (zero for ops that skip the channel)
  BatchOps ops;
};

// Every op is a spike and no two touch (same or conjugate frequency in an overlapping channel).
bool point_program(const tb_sample_ops& s, int H, int W, int D);
size_t point_workspace_bytes(int H, int bc);
hipError_t launch_point(const PointArgs& a, hipStream_t st, int stage);  // stage 0: K, 1: Delta, 2: apply

}  // namespace tb
