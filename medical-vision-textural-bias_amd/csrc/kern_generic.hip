// kern_generic.hip -- direct-DFT fallback of the full-spectrum passes, for transform sizes the
// mixed-radix slab passes do not take: an axis length with a prime factor above 31, or a (W, D)
// slab whose half spectrum exceeds the LDS.  The reference's torch.fft.fftn takes any size
// (source_code/filters_and_operators.py:594-632); this path keeps that contract at O(n) work per
// coefficient and axis instead of raising.
//
// The spectrum is the FULL complex one, S[bc][h][w][d] (complex64), in two ping-pong buffers:
//   load x -> S0;  DFT along D, W, H (S0 -> S1 -> S0 -> S1);  op program on S1;  inverse DFT
//   along H, W, D (S1 -> S0 -> S1 -> S0);  y = Re(S0) / (H W D) with the zero D-padding and the
//   per-sample min/max keys.
// The op program is apply_ops (fft_core.h), the same symmetrised form the half-spectrum passes use:
// on a full Hermitian spectrum it keeps the spectrum Hermitian, so Re(IFFT) is the reference's
// `.real` exactly as on the half spectrum.
#include <hip/hip_runtime.h>

#include <cstring>

#include "kernels.h"

namespace tb {

namespace {

constexpr int NT_GEN = 256;

// One DFT along an axis: the volume is viewed as [A][n][Bi] and pencil q = (ao, bi) holds the n
// elements ao*n*Bi + bi + j*Bi.  A workgroup takes PW consecutive pencils: loads them and the
// twiddles into LDS (consecutive bi are adjacent in memory, so a tile load is coalesced; with Bi == 1
// a pencil is one contiguous row), then each output y[k] = sum_j s[j] w^(j k) is one thread's sum.
__global__ __launch_bounds__(NT_GEN) void k_gen_dft(const cf* __restrict__ in, cf* __restrict__ out,
                                                    const cf* __restrict__ tw, int n, int64_t A, int64_t Bi, int PW,
                                                    int inverse) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cf* twl = reinterpret_cast<cf*>(smem);
  cf* s = twl + n;  // [n][PW]
  const int tid = (int)threadIdx.x;
  const int64_t q0 = (int64_t)blockIdx.x * PW, nq = A * Bi;
  const int np = (nq - q0) < PW ? (int)(nq - q0) : PW;
  for (int j = tid; j < n; j += NT_GEN) {
    const cf w = tw[j];
    twl[j] = inverse ? conj(w) : w;  // exp(+-2 pi i j / n)
  }
  const int tot = n * PW;
  for (int idx = tid; idx < tot; idx += NT_GEN) {
    int p, j;
    if (Bi == 1) { p = idx / n; j = idx - p * n; }
    else { j = idx / PW; p = idx - j * PW; }
    cf v = mk(0.f, 0.f);
    if (p < np) {
      const int64_t q = q0 + p, ao = q / Bi, bi = q - ao * Bi;
      v = in[ao * n * Bi + bi + (int64_t)j * Bi];
    }
    s[j * PW + p] = v;
  }
  __syncthreads();
  for (int idx = tid; idx < tot; idx += NT_GEN) {
    int p, k;
    if (Bi == 1) { p = idx / n; k = idx - p * n; }
    else { k = idx / PW; p = idx - k * PW; }
    if (p >= np) continue;
    float ax = 0.f, ay = 0.f;
    int t = 0;  // (j k) mod n
    for (int j = 0; j < n; ++j) {
      const cf a = s[j * PW + p], w = twl[t];
      ax = fmaf(a.x, w.x, fmaf(-a.y, w.y, ax));
      ay = fmaf(a.x, w.y, fmaf(a.y, w.x, ay));
      t += k;
      t = t >= n ? t - n : t;
    }
    const int64_t q = q0 + p, ao = q / Bi, bi = q - ao * Bi;
    out[ao * n * Bi + bi + (int64_t)k * Bi] = mk(ax, ay);
  }
}

struct GenArgs {
  tb_plan_dev pl;
  const float* x;
  int64_t xsbc, xsh, xsw;
  float* y;
  int64_t ysbc, ysh, ysw;
  cf* S;
  int ypad, bc0, C, nbc;
  float scale;
  uint32_t* mm;
  double* out;
  BatchOps ops;
};

// x (any strides, contiguous D) -> S0 = (x, 0)
__global__ __launch_bounds__(NT_GEN) void k_gen_load(GenArgs) {
  const GenArgs& a = kargs<GenArgs>();
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int64_t n = (int64_t)H * W * D;
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const float* xb = a.x + (int64_t)bc * a.xsbc;
  cf* Sb = a.S + (int64_t)bcl * n;
  for (int64_t e = (int64_t)blockIdx.x * NT_GEN + threadIdx.x; e < n; e += (int64_t)gridDim.x * NT_GEN) {
    const int64_t hw = e / D, d = e - hw * D, h = hw / W, w = hw - h * W;
    Sb[e] = mk(xb[h * a.xsh + w * a.xsw + d], 0.f);
  }
}

// the sample's op program on every coefficient of the full spectrum (in place)
__global__ __launch_bounds__(NT_GEN) void k_gen_ops(GenArgs) {
  const GenArgs& a = kargs<GenArgs>();
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int64_t n = (int64_t)H * W * D;
  const int bcl = (int)blockIdx.y;
  const int s = bcl / a.C, chan = bcl - s * a.C;  // sample within the run (bc0 = first sample * C)
  const tb_sample_ops& so = a.ops.s[s];
  cf* Sb = a.S + (int64_t)bcl * n;
  for (int64_t e = (int64_t)blockIdx.x * NT_GEN + threadIdx.x; e < n; e += (int64_t)gridDim.x * NT_GEN) {
    const int64_t hw = e / D;
    const int kd = (int)(e - hw * D), kh = (int)(hw / W), kw = (int)(hw - (int64_t)kh * W);
    Sb[e] = apply_ops(so, chan, Sb[e], freq_col(kw, kd, W, D), kh, H);
  }
}

// sum of log(|ops(K)| + 1e-10) over the full spectrum (tb_kspace_logabs_sum_f32)
__global__ __launch_bounds__(NT_GEN) void k_gen_logabs(GenArgs) {
  const GenArgs& a = kargs<GenArgs>();
  __shared__ double red[NT_GEN / 64];
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int64_t n = (int64_t)H * W * D;
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const int s = bcl / a.C, chan = bcl - s * a.C;
  const tb_sample_ops& so = a.ops.s[s];
  const cf* Sb = a.S + (int64_t)bcl * n;
  double acc = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * NT_GEN + threadIdx.x; e < n; e += (int64_t)gridDim.x * NT_GEN) {
    const int64_t hw = e / D;
    const int kd = (int)(e - hw * D), kh = (int)(hw / W), kw = (int)(hw - (int64_t)kh * W);
    const cf v = apply_ops(so, chan, Sb[e], freq_col(kw, kd, W, D), kh, H);
    acc += (double)logf(f32_sqrt(v.x * v.x + v.y * v.y) + 1e-10f);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NT_GEN / 64; ++w) acc += red[w];
    atomicAdd(&a.out[bc], acc);
  }
}

// y = Re(S0) * scale, zero D-padding, per-sample min/max keys (one sample per block)
__global__ __launch_bounds__(NT_GEN) void k_gen_store(GenArgs) {
  const GenArgs& a = kargs<GenArgs>();
  __shared__ float red[2 * NT_GEN / 64];
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int len = D + a.ypad;
  const int64_t n = (int64_t)H * W * len;
  const int bcl = (int)blockIdx.y, bc = a.bc0 + bcl;
  const cf* Sb = a.S + (int64_t)bcl * H * W * D;
  float* yb = a.y + (int64_t)bc * a.ysbc;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int64_t e = (int64_t)blockIdx.x * NT_GEN + threadIdx.x; e < n; e += (int64_t)gridDim.x * NT_GEN) {
    const int64_t hw = e / len, d = e - hw * len, h = hw / W, w = hw - h * W;
    float v = 0.f;
    if (d < D) {
      v = Sb[hw * D + d].x * a.scale;
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
    yb[h * a.ysh + w * a.ysw + d] = v;
  }
  if (a.mm) block_minmax_atomic<NT_GEN>(lo, hi, red, a.mm + 2 * (bc / a.C));
}

unsigned gen_blocks(int64_t n) {
  const int64_t b = (n + NT_GEN * 4 - 1) / (NT_GEN * 4);
  return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

// one axis of every channel-volume of the run: [nbc * before][n][after]
hipError_t gen_axis(const cf* in, cf* out, const cf* tw, int n, int64_t A, int64_t Bi, bool inverse, hipStream_t st) {
  int PW = Bi == 1 ? 4 : 16;
  while (PW > 1 && (size_t)n * (PW + 1) * sizeof(cf) > 65536) PW >>= 1;
  const size_t lds = (size_t)n * (PW + 1) * sizeof(cf);
  if (lds > 163840) return hipErrorInvalidValue;
  hipError_t e = allow_lds(k_gen_dft, lds);
  if (e != hipSuccess) return e;
  const int64_t nq = A * Bi, nb = (nq + PW - 1) / PW;
  if (nb >= (1LL << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gen_dft, dim3((unsigned)nb), dim3(NT_GEN), lds, st, in, out, tw, n, A, Bi, PW, inverse ? 1 : 0);
  return hipGetLastError();
}

// forward DFT of the run's channel-volumes into S1 (= S0 + nbc H W D)
hipError_t gen_forward(GenArgs& a, hipStream_t st) {
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int64_t n = (int64_t)H * W * D;
  cf* S0 = a.S;
  cf* S1 = a.S + (int64_t)a.nbc * n;
  hipLaunchKernelGGL(k_gen_load, dim3(gen_blocks(n), a.nbc), dim3(NT_GEN), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = gen_axis(S0, S1, a.pl.tw[2], D, (int64_t)a.nbc * H * W, 1, false, st);
  if (e == hipSuccess) e = gen_axis(S1, S0, a.pl.tw[1], W, (int64_t)a.nbc * H, D, false, st);
  if (e == hipSuccess) e = gen_axis(S0, S1, a.pl.tw[0], H, a.nbc, (int64_t)W * D, false, st);
  return e;
}

}  // namespace

size_t gen_workspace_bytes(int H, int W, int D, int bc) { return (size_t)2 * bc * H * W * D * sizeof(cf); }

hipError_t launch_gen_filter(const GenLaunch& g, hipStream_t st) {
  GenArgs a;
  std::memset(&a, 0, sizeof(a));
  a.pl = g.pl;
  a.x = g.x;
  a.xsbc = g.xs[0]; a.xsh = g.xs[1]; a.xsw = g.xs[2];
  a.y = g.y;
  a.ysbc = g.ys[0]; a.ysh = g.ys[1]; a.ysw = g.ys[2];
  a.S = g.S;
  a.ypad = g.ypad;
  a.bc0 = g.bc0;
  a.C = g.C;
  a.nbc = g.nbc;
  a.scale = (float)(1.0 / ((double)g.pl.H * (double)g.pl.W * (double)g.pl.D));
  a.mm = g.mm;
  a.ops = *g.ops;
  const int H = a.pl.H, W = a.pl.W, D = a.pl.D;
  const int64_t n = (int64_t)H * W * D;
  cf* S0 = a.S;
  cf* S1 = a.S + (int64_t)a.nbc * n;
  hipError_t e = gen_forward(a, st);
  if (e != hipSuccess) return e;
  a.S = S1;
  hipLaunchKernelGGL(k_gen_ops, dim3(gen_blocks(n), a.nbc), dim3(NT_GEN), 0, st, a);
  e = hipGetLastError();
  if (e == hipSuccess) e = gen_axis(S1, S0, a.pl.tw[0], H, a.nbc, (int64_t)W * D, true, st);
  if (e == hipSuccess) e = gen_axis(S0, S1, a.pl.tw[1], W, (int64_t)a.nbc * H, D, true, st);
  if (e == hipSuccess) e = gen_axis(S1, S0, a.pl.tw[2], D, (int64_t)a.nbc * H * W, 1, true, st);
  if (e != hipSuccess) return e;
  a.S = S0;
  hipLaunchKernelGGL(k_gen_store, dim3(gen_blocks(n), a.nbc), dim3(NT_GEN), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gen_logabs(const GenLaunch& g, double* out, hipStream_t st) {
  GenArgs a;
  std::memset(&a, 0, sizeof(a));
  a.pl = g.pl;
  a.x = g.x;
  a.xsbc = g.xs[0]; a.xsh = g.xs[1]; a.xsw = g.xs[2];
  a.S = g.S;
  a.bc0 = g.bc0;
  a.C = g.C;
  a.nbc = g.nbc;
  a.out = out;
  a.ops = *g.ops;
  const int64_t n = (int64_t)a.pl.H * a.pl.W * a.pl.D;
  hipError_t e = gen_forward(a, st);
  if (e != hipSuccess) return e;
  a.S = g.S + (int64_t)a.nbc * n;
  hipLaunchKernelGGL(k_gen_logabs, dim3(gen_blocks(n), a.nbc), dim3(NT_GEN), 0, st, a);
  return hipGetLastError();
}

}  // namespace tb
