// plan_host.h -- host-side plan construction shared by the library and the test emulator:
// FFT factorisation per axis, twiddle tables, digit-reversal tables.
#pragma once

#include <cmath>
#include <vector>

#include "fft_core.h"

namespace tb {

// radix preference: fewest LDS round trips first; composites are in-register DFTs
static const int kRadixPref[] = {16, 15, 12, 10, 9, 8, 6, 5, 4, 3, 2, 7, 11, 13, 17, 19, 23, 29, 31};

inline bool factorize(int n, tb_axis& ax) {
  ax.n = n;
  ax.nst = 0;
  int m = n;
  while (m > 1) {
    bool found = false;
    for (int r : kRadixPref) {
      if (m % r == 0) {
        if (ax.nst >= TB_MAX_STAGES) return false;
        ax.radix[ax.nst++] = r;
        m /= r;
        found = true;
        break;
      }
    }
    if (!found) return false;
  }
  return n >= 1;
}

inline int max_radix(const tb_axis& ax) {
  int r = 1;
  for (int s = 0; s < ax.nst; ++s) r = ax.radix[s] > r ? ax.radix[s] : r;
  return r;
}

// tw[t] = exp(-2 pi i t / n), computed in double and rounded once
inline std::vector<cf> twiddles(int n) {
  std::vector<cf> t(n > 0 ? n : 1);
  for (int i = 0; i < n; ++i) {
    // exact symmetric reduction keeps the table's quarter/half points exact
    const double a = -2.0 * kPi * (double)i / (double)n;
    t[i] = mk((float)std::cos(a), (float)std::sin(a));
  }
  return t;
}

// frequency k -> slot of the DIF output
inline std::vector<int> digit_rev(const tb_axis& ax) {
  std::vector<int> out(ax.n);
  for (int k = 0; k < ax.n; ++k) {
    int pos = 0, kk = k, Ls = ax.n;
    for (int s = 0; s < ax.nst; ++s) {
      const int r = ax.radix[s];
      const int q = kk % r;
      kk /= r;
      Ls /= r;
      pos += q * Ls;
    }
    out[k] = pos;
  }
  return out;
}

inline std::vector<int> inverse_perm(const std::vector<int>& p) {
  std::vector<int> q(p.size());
  for (size_t i = 0; i < p.size(); ++i) q[p[i]] = (int)i;
  return q;
}

struct PlanTables {
  int H, W, D;
  tb_axis ax[3];
  std::vector<cf> tw[3];
  std::vector<int> rev_d, irev_h, irev_w;
};

inline int build_tables(int H, int W, int D, PlanTables& pt) {
  if (H < 1 || W < 1 || D < 1) return TB_ERR_INVALID_ARG;
  pt.H = H; pt.W = W; pt.D = D;
  const int n[3] = {H, W, D};
  for (int a = 0; a < 3; ++a) {
    if (!factorize(n[a], pt.ax[a])) return TB_ERR_UNSUPPORTED_SIZE;
    pt.tw[a] = twiddles(n[a]);
  }
  pt.rev_d = digit_rev(pt.ax[2]);
  pt.irev_h = inverse_perm(digit_rev(pt.ax[0]));
  pt.irev_w = inverse_perm(digit_rev(pt.ax[1]));
  return TB_OK;
}

}  // namespace tb
