// Host sanitizer run of the kernels' item functions (test infrastructure): the emulator
// (emu.cpp -- the same fft_core.h / slab_ct.h / kspace_ct.h / sap_core.h code the gfx950 kernels run)
// built as ONE executable with -fsanitize=address,undefined, so no sanitizer runtime has to be preloaded
// into Python.  Runs the full-spectrum passes on odd / even / prime / padded shapes with identity, disk,
// wrap and spike programs, the Philox stream, the S&P classes and the min/max keys; exits non-zero on any
// invariant violation (the sanitizers abort on their own findings).
#include "emu.cpp"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

namespace {

int fails = 0;
#define EXPECT(c, ...)                     \
  do {                                     \
    if (!(c)) {                            \
      std::fprintf(stderr, __VA_ARGS__);   \
      std::fprintf(stderr, "\n");          \
      ++fails;                             \
    }                                      \
  } while (0)

tb_op op_of(int kind) {
  tb_op o;
  std::memset(&o, 0, sizeof(o));
  o.kind = kind;
  o.chan = -1;
  return o;
}

// runs one program on B x C x H x W x D random data; returns max |y| and checks padding / min / max keys
double run(int H, int W, int D, int pad, int B, int C, const std::vector<tb_op>& prog, int use_ct, std::vector<float>* out,
           std::vector<float>* xin) {
  const int64_t n = (int64_t)H * W * D;
  std::vector<float> x((size_t)B * C * n);
  std::mt19937 g(1234 + H + W + D);
  std::normal_distribution<float> nd;
  for (auto& v : x) v = nd(g);
  const int Dp = D + pad;
  std::vector<float> y((size_t)B * C * H * W * Dp, -7.f);
  const int64_t xs[3] = {n, (int64_t)W * D, D}, ys[3] = {(int64_t)H * W * Dp, (int64_t)W * Dp, Dp};
  std::vector<tb_sample_ops> ops(B);
  for (auto& so : ops) {
    std::memset(&so, 0, sizeof(so));
    so.n = (int)prog.size();
    for (size_t i = 0; i < prog.size(); ++i) so.op[i] = prog[i];
  }
  std::vector<float> mm((size_t)2 * B);
  const int rc = tbemu_kspace_filter_f32(H, W, D, x.data(), xs, y.data(), ys, pad, B, C, ops.data(), mm.data(), 0, use_ct);
  EXPECT(rc == 0, "rc %d at %dx%dx%d", rc, H, W, D);
  double mx = 0.0;
  for (int b = 0; b < B; ++b) {
    float lo = INFINITY, hi = -INFINITY;
    for (int c = 0; c < C; ++c)
      for (int r = 0; r < H * W; ++r)
        for (int d = 0; d < Dp; ++d) {
          const float v = y[(((size_t)b * C + c) * H * W + r) * Dp + d];
          if (d >= D) {
            EXPECT(v == 0.f, "padding not zero at %dx%dx%d", H, W, D);
            continue;
          }
          EXPECT(std::isfinite(v), "non-finite output at %dx%dx%d", H, W, D);
          lo = std::fmin(lo, v);
          hi = std::fmax(hi, v);
          mx = std::fmax(mx, std::fabs((double)v));
        }
    EXPECT(mm[2 * b] == lo && mm[2 * b + 1] == hi, "min/max keys differ at %dx%dx%d", H, W, D);
  }
  if (out) *out = y;
  if (xin) *xin = x;
  return mx;
}

}  // namespace

int main() {
  const int shapes[][3] = {{8, 6, 5}, {12, 10, 9}, {7, 11, 13}, {16, 16, 16}, {6, 4, 31}, {9, 8, 2}};
  for (const auto& s : shapes) {
    const int H = s[0], W = s[1], D = s[2];
    for (int pad : {0, 3}) {
      std::vector<float> y, x;
      run(H, W, D, pad, 2, 3, {}, 0, &y, &x);  // identity: y == x
      const int Dp = D + pad;
      double err = 0.0, ref = 0.0;
      for (size_t bc = 0; bc < 6; ++bc)
        for (int r = 0; r < H * W; ++r)
          for (int d = 0; d < D; ++d) {
            const double a = y[(bc * H * W + r) * Dp + d], b = x[(bc * H * W + r) * D + d];
            err = std::fmax(err, std::fabs(a - b));
            ref = std::fmax(ref, std::fabs(b));
          }
      EXPECT(err <= 2e-5 * ref, "identity error %g at %dx%dx%d pad %d", err / ref, H, W, D, pad);
      tb_op disk = op_of(TB_OP_DISK), wrap = op_of(TB_OP_WRAP), spike = op_of(TB_OP_SPIKE);
      disk.f[0] = 2.5f * 2.5f;
      wrap.f[0] = 0.5f;
      spike.i[0] = 1, spike.i[1] = 2 % W, spike.i[2] = 1 % D;
      spike.f[0] = 3.0f;
      run(H, W, D, pad, 2, 3, {disk, spike, wrap}, 0, nullptr, nullptr);
    }
  }
  // compiled slab plan shapes through the ct item functions (one small batch)
  {
    tb_op disk = op_of(TB_OP_DISK);
    disk.f[0] = 6.5f * 6.5f;
    run(16, 128, 64, 0, 1, 1, {disk}, 1, nullptr, nullptr);
  }
  // Philox stream, S&P classes, order-preserving keys
  std::vector<float> u(4099);
  tbemu_philox_u01(7, (int64_t)u.size(), 3, 99, u.data());
  for (float v : u) EXPECT(v >= 0.f && v < 1.f, "u01 out of range");
  std::vector<int8_t> cls(u.size());
  tbemu_sap_class(u.data(), (int64_t)u.size(), 0.05f, 0.1f, cls.data());
  for (size_t i = 0; i < u.size(); ++i)
    EXPECT(cls[i] == (u[i] <= 0.05f ? 1 : (u[i] <= 0.1f ? 2 : 0)), "class %zu", i);
  for (float f : {-3.5f, -0.f, 0.f, 1e-30f, 7.25f, -INFINITY, INFINITY})
    EXPECT(tbemu_key2f(tbemu_f2key(f)) == f, "key round trip %g", f);
  EXPECT(tbemu_f2key(-1.f) < tbemu_f2key(1.f), "key order");
  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("emu sanitizer run ok\n");
  return 0;
}
