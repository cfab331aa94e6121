// texbias.hip -- gfx950 kernels and the C ABI (include/texbias.h) of the texbias library.
//
// The pass kernels A/B/C (and the spectrum statistics) live in kern_*.hip, one translation unit
// per kernel and radix set; this file holds the small kernels and the host side of the C ABI.
// Pass plan of one k-space filter call (DESIGN.md "Kernels"):
//   A  k_slab_fwd   per (bc, h) slab: real rows -> pair-packed R2C along D -> C2C along W,
//                   in one 150 KB LDS slab; stores the half spectrum (digit-reversed W).
//   B  k_kspace     per (bc, tile of T spectrum columns): C2C along H (DIF), the sample's
//                   op program on every coefficient, inverse along H (DIT).
//   C  k_slab_inv   per (bc, h) slab: inverse W, C2R along D, scale 1/N, zero D-padding,
//                   per-sample min/max epilogue.
//   D  k_salt_pepper  Philox u, class, sparse in-place MIN/MAX scatter.
#include <hip/hip_runtime.h>

#include <cmath>
#include <math.h>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "band.h"
#include "fft_core.h"
#include "kernels.h"
#include "point.h"
#include "plan_host.h"
#include "sap_core.h"
#include "wrap.h"

using namespace tb;

namespace {

thread_local int g_last_hip = 0;
// compiled (compile-time) plans enabled: TEXBIAS_COMPILED_PLANS=0 or tb_set_compiled_plans(0) turns
// them off, e.g. to compare against the generic passes
bool g_compiled_plans = [] {
  const char* e = std::getenv("TEXBIAS_COMPILED_PLANS");
  return !(e && e[0] == '0');
}();

inline int hip_fail(hipError_t e) {
  g_last_hip = (int)e;
  return TB_ERR_HIP;
}
#define TB_HIP(call)                              \
  do {                                            \
    hipError_t e_ = (call);                       \
    if (e_ != hipSuccess) return hip_fail(e_);    \
  } while (0)

// ------------------------------------------------------------------ timing
struct TimingRec {
  hipEvent_t a, b;
  int slot;
  double bytes;
};
std::mutex g_tmu;
bool g_timing = false;
std::vector<TimingRec> g_recs;
std::vector<hipEvent_t> g_pool;
const char* g_slot_kernel[4] = {"", "", "", ""};

hipEvent_t ev_get() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  // Timing-only events: no system-scope release / acquire around the pass (hipEventDisableSystemFence),
  // so the end stamp is not delayed by an L2 write-back and the pass does not start on invalidated
  // caches -- the stamps bracket the kernel itself (round 6: every pass 1-2 us shorter than with
  // default events, which rocprofv3's kernel durations confirm).
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}
struct Timer {  // records [begin, end) of one pass when timing is enabled
  hipEvent_t a = nullptr, b = nullptr;
  int slot;
  double bytes;
  hipStream_t st;
  // bytes: the launch's algorithmic HBM bytes (each global input/output element counted once)
  Timer(int s, hipStream_t stream, double nbytes = 0.0, const char* kernel = nullptr)
      : slot(s), bytes(nbytes), st(stream) {
    if (!g_timing) return;
    std::lock_guard<std::mutex> lk(g_tmu);
    if (kernel) g_slot_kernel[s] = kernel;
    a = ev_get();
    b = ev_get();
    if (a) (void)hipEventRecord(a, st);
  }
  ~Timer() {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    std::lock_guard<std::mutex> lk(g_tmu);
    g_recs.push_back({a, b, slot, bytes});
  }
};

// ---------------------------------------------------------------- kernels

__global__ void k_minmax_init(uint32_t* mm, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    mm[2 * i] = 0xffffffffu;
    mm[2 * i + 1] = 0u;
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_minmax(const float* __restrict__ x, uint32_t* __restrict__ mm, int64_t rows,
                                               int len, int64_t ld, int64_t sb) {
  __shared__ float red[2 * NT / 64];
  const int b = blockIdx.y;
  const float* xb = x + b * sb;
  const int64_t n = rows * len;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / len;
    const float v = xb[r * ld + (i - r * len)];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  block_minmax_atomic<NT>(lo, hi, red, mm + 2 * b);
}

struct SapThr {
  float lo[TB_MAX_BATCH], hi[TB_MAX_BATCH];
};

template <int NT>
__global__ __launch_bounds__(NT) void k_salt_pepper(const float* __restrict__ x, float* __restrict__ y,
                                                    int8_t* __restrict__ cls, const float* __restrict__ uin,
                                                    uint64_t seed, uint64_t offset, SapThr thr,
                                                    const uint32_t* __restrict__ mm, int b0, int64_t rows, int len,
                                                    int64_t ld, int64_t sb, int sparse) {
  const int bl = blockIdx.y;
  const int b = b0 + bl;
  const int64_t n = rows * len;
  const float vmin = key2f(mm[2 * b]) * 0.5f, vmax = key2f(mm[2 * b + 1]) * 0.5f;
  const float lo = thr.lo[bl], hi = thr.hi[bl];
  const int64_t lin0 = (int64_t)b * n;  // logical (unpadded) voxel index of this sample
  const int64_t ngroups = (n + 3) / 4;
  for (int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x; g < ngroups; g += (int64_t)gridDim.x * NT) {
    u32x4 r;
    if (!uin) r = philox((uint64_t)(lin0 / 4 + g), offset, seed);  // n % 4 handled below
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i = 4 * g + q;
      if (i >= n) break;
      // element offset of voxel i; 32-bit division while the sample fits (the 64-bit one is ~4x the
      // VALU work), and in the sparse Philox path only for the ~p of voxels that are written
      auto offset_of = [&]() -> int64_t {
        const int64_t row = n < 0x7fffffff ? (int64_t)((uint32_t)i / (uint32_t)len) : i / len;
        return b * sb + row * ld + (i - row * len);
      };
      float u;
      int64_t off = -1;
      if (uin) {
        off = offset_of();
        u = uin[off];
      } else {
        // counter of logical voxel L = lin0 + i: the group index and lane of L itself, so the
        // stream is independent of how samples are batched when n % 4 == 0 (the usual case)
        if ((lin0 & 3) == 0) u = u01(r.v[q]);
        else {
          const int64_t L = lin0 + i;
          u = u01(philox((uint64_t)(L >> 2), offset, seed).v[L & 3]);
        }
      }
      const int c = sap_class(u, lo, hi);
      if (cls || !sparse || c) {
        if (off < 0) off = offset_of();
        if (cls) cls[off] = (int8_t)c;
        if (sparse) {
          if (c) y[off] = c == 1 ? vmin : vmax;
        } else {
          y[off] = c == 0 ? x[off] : (c == 1 ? vmin : vmax);
        }
      }
    }
  }
}

// Salt-and-pepper from the device stream: instead of one uniform per voxel, each lane walks a
// segment of SAP_SEG voxels jumping straight to the next changed voxel -- the gap to it is
// geometric, floor(log(u) / log(1 - p)) -- and draws its class (MIN with probability lo / hi).
// The changed voxels form the same Bernoulli(p) field with P(MIN) = p_lo, P(MAX) = p_hi - p_lo
// as u <= lo / lo < u <= hi of the reference (:478-479), at ~p of the RNG work.
#ifndef TB_SAP_SEG
#define TB_SAP_SEG 256  // voxels per thread: 4 waves per SIMD on a C3 launch (1024: 61 us, 256: 51.5 us;
                        // blocks walking the volume last to first, where the previous pass's last lines
                        // might still be cached: no change, 48.2 vs 48.5 us; round 6: the same walk into
                        // a per-wave LDS bitmap, then stored in address order with one masked store per
                        // 64 voxels -- half the L2 requests -- 78 vs 48 us, dropped)
#endif
constexpr int SAP_SEG = TB_SAP_SEG;
struct SapGeomArgs {
  float* y;
  int8_t* cls;
  uint64_t seed, offset;
  float lo[TB_MAX_BATCH], hi[TB_MAX_BATCH];
  const uint32_t* mm;
  int b0;
  int64_t rows;
  int len;
  int64_t ld, sb;
};
__global__ __launch_bounds__(256) void k_sap_geom(SapGeomArgs a) {
  const int bl = blockIdx.y, b = a.b0 + bl;
  const int64_t n = a.rows * a.len;
  const int64_t start = ((int64_t)blockIdx.x * 256 + threadIdx.x) * SAP_SEG;
  const float p = a.hi[bl];
  if (start >= n || !(p > 0.f)) return;
  const int64_t end = start + SAP_SEG < n ? start + SAP_SEG : n;
  const float vmin = key2f(a.mm[2 * b]) * 0.5f, vmax = key2f(a.mm[2 * b + 1]) * 0.5f;
  const float pmin = a.lo[bl] > 0.f ? a.lo[bl] / p : 0.f;  // P(MIN | changed)
  const float lq = p >= 1.f ? -INFINITY : log1pf(-p);
  const uint64_t ctr0 = ((uint64_t)b << 44) ^ ((uint64_t)(start / SAP_SEG) << 20);
  int64_t pos = start - 1;
  uint32_t j = 0;
  for (;;) {
    const u32x4 r = philox(ctr0 | j++, a.offset, a.seed);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float u1 = ((float)(r.v[2 * h] >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
      const float g = lq == -INFINITY ? 0.f : floorf(logf(u1) / lq);
      pos += 1 + (g < (float)SAP_SEG ? (int64_t)g : (int64_t)SAP_SEG);
      if (pos >= end) return;
      const int c = u01(r.v[2 * h + 1]) < pmin ? 1 : 2;
      const int64_t row = n < 0x7fffffff ? (int64_t)((uint32_t)pos / (uint32_t)a.len) : pos / a.len;
      const int64_t off = b * a.sb + row * a.ld + (pos - row * a.len);
      a.y[off] = c == 1 ? vmin : vmax;
      if (a.cls) a.cls[off] = (int8_t)c;
    }
  }
}

__global__ void k_disk_mask(float* __restrict__ m, int64_t outer, int n0, int n1, int n2, int int_r, int64_t r2i,
                            float r2f, int inside_off) {
  const int64_t per = (int64_t)n0 * n1 * n2;
  const int64_t total = outer * per;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i % per;
    const int i2 = (int)(r % n2);
    r /= n2;
    const int i1 = (int)(r % n1);
    const int i0 = (int)(r / n1);
    const int64_t d0 = i0 - n0 / 2, d1 = i1 - n1 / 2, d2 = i2 - n2 / 2;
    const int64_t s = d0 * d0 + d1 * d1 + d2 * d2;
    bool in = int_r ? (s < r2i) : ((float)s < r2f);
    if (inside_off) in = !in;
    m[i] = in ? 1.f : 0.f;
  }
}

}  // namespace

// ------------------------------------------------------------------- plan
struct tb_plan {
  tb_plan_dev dev;
  PlanTables host;
  void* dmem = nullptr;
  int rset_h = RS_ALL;   // radix set of the H axis (pass B)
  int rset_wd = RS_ALL;  // radix set of the W and D axes (passes A, C)
  int lds_max = 65536;
  int ncu = 256;         // compute units (grid of the persistent compiled-plan slab kernels)
  bool ct_slab = false;  // (W, D) has a compile-time slab plan (slab_ct.h)
  bool ct_tile = false;  // H has a compile-time pass-B plan (kspace_ct.h)
  bool ct_half = false;  // (H, W, D) has half-unit passes A / C and the split pass B (slab_ct.h HalfPlan)
  float* tds = nullptr;  // band pass C': [D/2 + 1][2][NCOLS] cos / sin(2 pi kd d / D), d < D/2 + 1, else 0
  float* tbt = nullptr;  // band pass A': [2][KSd][2][64] B fragments of the folded D product
  void* tbt16 = nullptr;  // band pass A', compiled D: split-f16 B fragments [KS16][cos/sin][hi/lo][64][8]
  bool generic = false;  // full-spectrum route on the direct-DFT fallback (kern_generic.hip)
  double* wrapq = nullptr;  // odd D <= WRAP_MAX_COLS: the wrap route's D circulant table q[D] (wrap.h)
};

namespace {

constexpr int NT_SAP = 256;

bool needs_all(const tb_axis& ax) {
  for (int s = 0; s < ax.nst; ++s) {
    const int r = ax.radix[s];
    if (r > 10 && r != 12 && r != 15 && r != 16) return true;
  }
  return false;
}

int pick_tile(int H, int lds_max) {
  // ~32 KB tiles (measured best of 16/32/64 KB at H = 240: 4 workgroups per CU, 128-B rows)
  constexpr int budget = 32768;
  int T = budget / (H * 8);
  if (T > 64) T = 64;
  if (T >= 16) T &= ~7;   // whole 64-B segments per tile row
  if (T < 4) T = 4;
  while (tile_geo(H, T).total_cf * 8 > lds_max && T > 1) --T;
  return T;
}

}  // namespace

// Exported functions: C linkage comes from their declarations in texbias.h.
int tb_version(void) { return TB_VERSION; }

const char* tb_error_string(int code) {
  switch (code) {
    case TB_OK: return "ok";
    case TB_ERR_INVALID_ARG: return "invalid argument";
    case TB_ERR_UNSUPPORTED_SIZE: return "unsupported transform size (an axis above the direct-DFT fallback's 10240)";
    case TB_ERR_HIP: return "HIP runtime error";
    case TB_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown error";
  }
}

int tb_last_hip_error(void) { return g_last_hip; }

int tb_plan_create(int H, int W, int D, tb_plan** out) {
  if (!out) return TB_ERR_INVALID_ARG;
  *out = nullptr;
  tb_plan* p = new tb_plan();
  int rc = build_tables(H, W, D, p->host);
  if (rc == TB_ERR_UNSUPPORTED_SIZE) {
    // an axis with a prime factor > 31: the full-spectrum route runs on the direct-DFT fallback
    // (the band passes take any size); the mixed-radix tables are never read
    p->generic = true;
    const int n[3] = {H, W, D};
    for (int a = 0; a < 3; ++a) {
      if (!factorize(n[a], p->host.ax[a])) {
        p->host.ax[a].n = n[a];
        p->host.ax[a].nst = 0;
      }
      p->host.tw[a] = twiddles(n[a]);
    }
    p->host.rev_d.resize(D);
    p->host.irev_h.resize(H);
    p->host.irev_w.resize(W);
    for (int i = 0; i < D; ++i) p->host.rev_d[i] = i;
    for (int i = 0; i < H; ++i) p->host.irev_h[i] = i;
    for (int i = 0; i < W; ++i) p->host.irev_w[i] = i;
  } else if (rc != TB_OK) {
    delete p;
    return rc;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { delete p; return hip_fail(hipGetLastError()); }
  int lds = 0;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess && lds > 0)
    p->lds_max = lds;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
    p->ncu = ncu;
  // compile-time slab plan: same shape and therefore the same radix order as the runtime plan
  p->ct_slab = !p->generic && tb::slab_ct_supported(W, D);
  p->ct_tile = !p->generic && tb::kspace_ct_supported(H);
  p->ct_half = !p->generic && tb::slab_half_supported(W, D) && tb::kspace_half_supported(H, W, D);
  const SlabGeo sg = slab_geo(W, D);
  if ((size_t)sg.total_cf * 8 > (size_t)p->lds_max) p->generic = true;  // slab above the LDS: fallback too
  if (p->generic) p->ct_slab = p->ct_half = false;
  // device tables: tw[H], tw[W], tw[D] (cf) + rev_d[D], irev_h[H], irev_w[W] (int)
  const size_t ncf = (size_t)H + W + D, nint = (size_t)D + H + W;
  const size_t bytes = ncf * sizeof(cf) + nint * sizeof(int);
  std::vector<char> buf(bytes);
  char* q = buf.data();
  size_t off_tw[3], off_i[3];
  size_t o = 0;
  const int n[3] = {H, W, D};
  for (int a = 0; a < 3; ++a) {
    off_tw[a] = o;
    std::memcpy(q + o, p->host.tw[a].data(), n[a] * sizeof(cf));
    o += n[a] * sizeof(cf);
  }
  const std::vector<int>* iv[3] = {&p->host.rev_d, &p->host.irev_h, &p->host.irev_w};
  for (int a = 0; a < 3; ++a) {
    off_i[a] = o;
    std::memcpy(q + o, iv[a]->data(), iv[a]->size() * sizeof(int));
    o += iv[a]->size() * sizeof(int);
  }
  if (hipMalloc(&p->dmem, bytes) != hipSuccess) { delete p; return hip_fail(hipGetLastError()); }
  if (hipMemcpy(p->dmem, buf.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(p->dmem);
    delete p;
    return hip_fail(hipGetLastError());
  }
  char* d = static_cast<char*>(p->dmem);
  p->dev.H = H; p->dev.W = W; p->dev.D = D; p->dev.pad = 0;
  for (int a = 0; a < 3; ++a) {
    p->dev.ax[a] = p->host.ax[a];
    p->dev.tw[a] = reinterpret_cast<const cf*>(d + off_tw[a]);
  }
  p->dev.rev_d = reinterpret_cast<const int*>(d + off_i[0]);
  p->dev.irev_h = reinterpret_cast<const int*>(d + off_i[1]);
  p->dev.irev_w = reinterpret_cast<const int*>(d + off_i[2]);
  if (D <= BAND_MAX_D) {  // folded synthesis table (pass C') and the D-product B fragments (pass A'),
                         // double precision; plans no band route can take (D > BAND_MAX_D) skip them
    const int Dh = D / 2 + 1, ncols = 32 * ((Dh + 31) / 32), KSd = (Dh + 3) / 4;
    std::vector<float> ts((size_t)Dh * 2 * ncols, 0.f), tb((size_t)2 * KSd * 2 * 64, 0.f);
    for (int k = 0; k < Dh; ++k)
      for (int d = 0; d < Dh; ++d) {
        const double ang = 2.0 * 3.14159265358979323846 * (double)(((int64_t)k * d) % D) / (double)D;
        ts[((size_t)k * 2) * ncols + d] = (float)std::cos(ang);
        ts[((size_t)k * 2 + 1) * ncols + d] = (float)std::sin(ang);
      }
    for (int nt = 0; nt < 2; ++nt)
      for (int ks = 0; ks < KSd; ++ks)
        for (int part = 0; part < 2; ++part)
          for (int ln = 0; ln < 64; ++ln) {
            const int d = 4 * ks + (ln >> 4), kd = 16 * nt + (ln & 15);
            if (d >= Dh || kd >= Dh) continue;
            const double ang = 2.0 * 3.14159265358979323846 * (double)(((int64_t)kd * d) % D) / (double)D;
            tb[(((size_t)nt * KSd + ks) * 2 + part) * 64 + ln] = (float)(part ? std::sin(ang) : std::cos(ang));
          }
    if (D == 155) {  // the compiled pass-A' kernel's split-f16 table (x 2^8, hi / lo halves)
      const int KS16 = tb::band_fwd16_ks(D);
      std::vector<_Float16> t16((size_t)KS16 * 2 * 2 * 64 * 8);
      for (int ks = 0; ks < KS16; ++ks)
        for (int part = 0; part < 2; ++part)
          for (int ln = 0; ln < 64; ++ln)
            for (int i = 0; i < 8; ++i) {  // B[k = 8 (ln / 16) + i][n = ln % 16]: folded d, kd
              const int d = 32 * ks + 8 * (ln >> 4) + i, kd = ln & 15;
              double v = 0.0;
              if (d < Dh && kd < Dh) {
                const double ang = 2.0 * 3.14159265358979323846 * (double)(((int64_t)kd * d) % D) / (double)D;
                v = (part ? std::sin(ang) : std::cos(ang)) * (double)tb::BAND_FWD16_TSCALE;
              }
              const float vf = (float)v;
              const _Float16 h = (_Float16)vf, l = (_Float16)(vf - (float)h);
              t16[((((size_t)ks * 2 + part) * 2 + 0) * 64 + ln) * 8 + i] = h;
              t16[((((size_t)ks * 2 + part) * 2 + 1) * 64 + ln) * 8 + i] = l;
            }
      if (hipMalloc(&p->tbt16, t16.size() * 2) != hipSuccess ||
          hipMemcpy(p->tbt16, t16.data(), t16.size() * 2, hipMemcpyHostToDevice) != hipSuccess) {
        tb_plan_destroy(p);
        return hip_fail(hipGetLastError());
      }
    }
    if (hipMalloc(reinterpret_cast<void**>(&p->tds), ts.size() * 4) != hipSuccess ||
        hipMemcpy(p->tds, ts.data(), ts.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&p->tbt), tb.size() * 4) != hipSuccess ||
        hipMemcpy(p->tbt, tb.data(), tb.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      tb_plan_destroy(p);
      return hip_fail(hipGetLastError());
    }
  }
  if ((D & 1) && D <= WRAP_MAX_COLS) {  // separable wrap route's D-axis circulant (float64)
    std::vector<double> q(D);
    tb::wrap_q_table(D, q.data());
    if (hipMalloc(reinterpret_cast<void**>(&p->wrapq), q.size() * 8) != hipSuccess ||
        hipMemcpy(p->wrapq, q.data(), q.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
      tb_plan_destroy(p);
      return hip_fail(hipGetLastError());
    }
  }
  p->rset_h = needs_all(p->host.ax[0]) ? RS_ALL : RS_SMALL;
  p->rset_wd = (needs_all(p->host.ax[1]) || needs_all(p->host.ax[2])) ? RS_ALL : RS_SMALL;
  *out = p;
  return TB_OK;
}

int tb_plan_destroy(tb_plan* plan) {
  if (!plan) return TB_OK;
  if (plan->dmem) (void)hipFree(plan->dmem);
  if (plan->tds) (void)hipFree(plan->tds);
  if (plan->tbt) (void)hipFree(plan->tbt);
  if (plan->tbt16) (void)hipFree(plan->tbt16);
  if (plan->wrapq) (void)hipFree(plan->wrapq);
  delete plan;
  return TB_OK;
}

size_t tb_workspace_bytes(const tb_plan* plan, int bc) {
  if (!plan || bc < 0) return 0;
  const size_t spec = (size_t)bc * plan->dev.H * plan->dev.W * (plan->dev.D / 2 + 1) * sizeof(cf);
  // the band passes' largest layout (band_plan() refuses boxes past these limits)
  BandGeo g{};
  g.KH = BAND_MAX_KH;
  g.KW = 31;
  g.NDk = BAND_MAX_NDK;
  g.ncol = BAND_MAX_ZCOL;
  g.KS = 32;
  g.NCOL = 32 * ((plan->dev.D / 2 + 1 + 31) / 32);
  g.cat = 0;  // 2 KS = 64 rows: the most either layout uses
  g.PT = 0;
  g.NTD = (plan->dev.D + 31) / 32 + 64;  // the split-f16 table for any pad up to 2048 columns
  const size_t band = band_ws(g, plan->dev.H, bc).total;
  const size_t gen = plan->generic ? gen_workspace_bytes(plan->dev.H, plan->dev.W, plan->dev.D, bc) : 0;
  const size_t m = spec > band ? spec : band;
  return m > gen ? m : gen;
}

int tb_plan_radices(const tb_plan* plan, int axis, int* radices) {
  if (!plan || axis < 0 || axis > 2 || !radices) return -1;
  const tb_axis& a = plan->dev.ax[axis];
  for (int s = 0; s < a.nst; ++s) radices[s] = a.radix[s];
  return a.nst;
}

static bool use_ct_slab(const tb_plan* p) { return g_compiled_plans && p->ct_slab; }

// Half units + split spectrum for the full route's passes (slab_ct.h HalfPlan) where the plan has
// them; TEXBIAS_HALF=0 or tb_set_half_units(0): the whole-slab compiled passes.
static bool g_half = [] {
  const char* e = std::getenv("TEXBIAS_HALF");
  return !(e && e[0] == '0');
}();
static bool use_half(const tb_plan* p) { return g_half && g_compiled_plans && p->ct_half; }

// channel-volumes per A -> B -> C chain (tb_set_chain_chunk; 0 = all, the default).  Chunks of
// 2..4 channel-volumes keep the spectrum within the Infinity Cache between passes, but measured
// slower at C3 (0.99 / 0.94 / 0.89 vs 0.85 ms per step: the passes are latency-bound, not
// HBM-bound, and smaller launches leave more of the chip idle in their tails).
static int g_chunk = -1;  // tb_set_chain_chunk
static int chunk_bc(const tb_plan*) { return g_chunk > 0 ? g_chunk : 0; }

template <int RS>
static int launch_slab_fwd(const tb_plan* p, const float* x, const int64_t* xs, cf* S, int bc0, int nbc,
                           hipStream_t st) {
  SlabFwdArgs a{p->dev, x, xs[0], xs[1], xs[2], S, bc0, nbc};
  if (use_ct_slab(p)) {
    TB_HIP(tb::launch_slab_fwd_ct(a, p->ncu, st));
    return TB_OK;
  }
  const size_t lds = (size_t)slab_geo(p->dev.W, p->dev.D).total_cf * sizeof(cf);
  TB_HIP(tb::launch_slab_fwd<RS>(a, dim3(p->dev.H, nbc), lds, st));
  return TB_OK;
}

// ------------------------------------------------------------ band-limited plans (band.h)
// TEXBIAS_BAND=0 or tb_set_band_plans(0) forces the full-spectrum passes for every program.
static bool g_band = [] {
  const char* e = std::getenv("TEXBIAS_BAND");
  return !(e && e[0] == '0');
}();
// Spike-only programs (plane waves, k-space spikes) in closed form (point.h); TEXBIAS_POINT=0 or
// tb_set_point_plans(0): the full-spectrum passes.
static bool g_point = [] {
  const char* e = std::getenv("TEXBIAS_POINT");
  return !(e && e[0] == '0');
}();
// Wrap-only programs on the separable route (wrap.h); TEXBIAS_WRAP=0 or tb_set_wrap_plans(0): the
// full-spectrum passes.
static bool g_wrap = [] {
  const char* e = std::getenv("TEXBIAS_WRAP");
  return !(e && e[0] == '0');
}();
// Pass C' synthesis in split f16 on the matrix cores (k_band_inv16) when the launch's V rows fit
// (band columns + every sample's points <= 64); TEXBIAS_INV16=0 or tb_set_band_inv16(0): the f32 kernel.
static bool g_inv16 = [] {
  const char* e = std::getenv("TEXBIAS_INV16");
  return !(e && e[0] == '0');
}();
// measurement only: TEXBIAS_BAND_DIAG=0xIIFF skips stages of A' (FF) / C' (II); results invalid
static int g_band_diag = [] {
  const char* e = std::getenv("TEXBIAS_BAND_DIAG");
  return e ? (int)std::strtol(e, nullptr, 0) : 0;
}();

// A low-pass op that zeroes every coefficient outside a box around DC (all channels).
static bool band_is_lowpass(const tb_op& op) {
  if (op.chan != -1) return false;
  if (op.kind == TB_OP_DISK) return op.i[1] == 0;       // inside_off = False: keeps the disk
  if (op.kind == TB_OP_GIBBS) return true;
  if (op.kind == TB_OP_LAYER) return op.l == 0;          // alpha known on the host
  return false;
}
// The op's own keep-test on a total squared distance (apply_ops' arithmetic, fft_core.h).
static bool band_keeps(const tb_op& op, int64_t sq) {
  if (op.kind == TB_OP_DISK) return op.i[0] ? (sq < op.l) : ((float)sq < op.f[0]);
  if (op.kind == TB_OP_GIBBS) return sq <= op.l;
  return layer_in(op, (int)sq);
}
// Largest |signed frequency| on an axis of length n that the op can keep, the other axes at their
// smallest term `rest` (disk: 0; Gibbs / layer: 0 for odd n, 1 for even n -- the (n-1)/2 centre);
// `half`: the D axis, stored kd in [0, n/2] only.  -1 when no coefficient survives.
static int band_extent(const tb_op& op, int n, int64_t rest, bool half) {
  int K = -1;
  const int kmax = half ? n / 2 : n - 1;
  for (int k = 0; k <= kmax; ++k) {
    const AxisGeo g = axis_geo(k, n);
    const int64_t term = op.kind == TB_OP_DISK ? g.dsq : (g.ef < g.en ? g.ef : g.en);
    if (!band_keeps(op, term + rest)) continue;
    const int m = (half || k <= (n - 1) / 2) ? k : n - k;
    K = m > K ? m : K;
  }
  return K;
}
static int band_minterm(const tb_op& op, int n) { return (op.kind == TB_OP_DISK || (n & 1)) ? 0 : 1; }

// Box of one sample's program (false: no low-pass, the full passes run).
static bool band_box(const tb_sample_ops& so, int H, int W, int D, int& KH, int& KW, int& KD) {
  for (int o = 0; o < so.n; ++o) {
    const tb_op& op = so.op[o];
    if (!band_is_lowpass(op)) continue;
    const int mh = band_minterm(op, H), mw = band_minterm(op, W), md = band_minterm(op, D);
    KH = band_extent(op, H, mw + md, false);
    KW = band_extent(op, W, mh + md, false);
    KD = band_extent(op, D, mh + mw, true);
    if (KH < 0 || KW < 0 || KD < 0) KH = KW = KD = 0;  // nothing kept: the box degenerates to DC
    return true;
  }
  return false;
}
// Stored (kd <= D/2) coefficients of the program's spikes that fall outside the box.
static bool band_points(const tb_sample_ops& so, int H, int W, int D, int KH, int KW, int KD, BandSamplePts& sp) {
  sp.n = 0;
  for (int o = 0; o < so.n; ++o) {
    const tb_op& op = so.op[o];
    if (op.kind != TB_OP_SPIKE) continue;
    const int f[2][3] = {{op.i[0], op.i[1], op.i[2]},
                         {(H - op.i[0]) % H, (W - op.i[1]) % W, (D - op.i[2]) % D}};
    for (int q = 0; q < 2; ++q) {
      const int kh = f[q][0], kw = f[q][1], kd = f[q][2];
      if (kd > D / 2) continue;
      const int mh = kh <= (H - 1) / 2 ? kh : H - kh, mw = kw <= (W - 1) / 2 ? kw : W - kw;
      if (mh <= KH && mw <= KW && kd <= KD) continue;  // inside the box: handled by pass B'
      bool dup = false;
      for (int j = 0; j < sp.n; ++j) dup |= sp.p[j].kh == kh && sp.p[j].kw == kw && sp.p[j].kd == kd;
      if (dup) continue;
      if (sp.n == BAND_MAX_PTS) return false;
      sp.p[sp.n].kh = (int16_t)kh;
      sp.p[sp.n].kw = (int16_t)kw;
      sp.p[sp.n].kd = (int16_t)kd;
      sp.p[sp.n].pad = 0;
      ++sp.n;
    }
  }
  return true;
}

// Band geometry shared by samples [s0, s1) of `ops`, or false when the run must use the full passes.
static bool band_plan(const tb_plan* p, const tb_sample_ops* ops, int s0, int s1, int y_pad, size_t ws_bytes, int bcn,
                      BandGeo& g, BandSamplePts* sp) {
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  int KH = 0, KW = 0, KD = 0, npt = 0;
  for (int s = s0; s < s1; ++s) {
    int kh, kw, kd;
    if (!band_box(ops[s], H, W, D, kh, kw, kd)) return false;
    KH = kh > KH ? kh : KH;
    KW = kw > KW ? kw : KW;
    KD = kd > KD ? kd : KD;
  }
  for (int s = s0; s < s1; ++s) {
    if (!band_points(ops[s], H, W, D, KH, KW, KD, sp[s - s0])) return false;
    npt = sp[s - s0].n > npt ? sp[s - s0].n : npt;
  }
  g.KH = KH;
  g.KW = KW;
  g.NDk = KD + 1;
  g.NW = 2 * KW + 1;
  g.ncol = g.NW * g.NDk;
  g.KS = g.NDk + npt;
  g.NCOL = 32 * ((D / 2 + 1 + 31) / 32);
  int ptot = 0;
  for (int s = s0; s < s1; ++s) ptot += sp[s - s0].n;
  g.cat = (g_inv16 && g.NDk + ptot <= 32) ? 1 : 0;
  g.PT = g.cat ? ptot : 0;
  g.NTD = (D + y_pad + 31) / 32;
  if (D > BAND_MAX_D || 2 * KH + 1 > H || 2 * KW + 1 > W || g.NDk > BAND_MAX_NDK || KW >= 32 || KH > BAND_MAX_KH)
    return false;
  if (g.ncol > BAND_MAX_ZCOL || W > 1024 || band_hc_lds(H, KH) > 160000) return false;
  if (2 * g.KS > 64 || g.KS > 32) return false;  // pass C' holds V in at most two 32-row MFMA tiles
  // worth it only when the box is a small part of the half spectrum
  if ((double)(2 * KH + 1) * g.ncol * 4.0 > (double)H * W * (D / 2 + 1)) return false;
  if (g.cat && band_inv16_carve(g, W).total > 160000) {
    g.cat = 0;
    g.PT = 0;
  }
  if (band_lds_fwd(g, W, D, false) > 160000 || band_lds_fwd(g, W, D, true) > 160000 ||
      (!g.cat && band_inv_carve(g, W, D).total > 160000))
    return false;
  if (band_ws(g, H, bcn).total > ws_bytes) return false;
  return true;
}

enum { RUN_COPY = 0, RUN_FULL = 1, RUN_BAND = 2, RUN_POINT = 3, RUN_WRAP = 4 };

// The run [s0, s1) takes the separable wrap route: every program wrap-only (with the same alpha
// product when D is odd: one circulant table per launch), a shape the route takes, room for its partials.
static bool wrap_run(const tb_plan* p, const tb_sample_ops* ops, int s, int y_pad, size_t ws_bytes, float* alpha) {
  if (!g_wrap || ws_bytes < tb::wrap_ws_bytes()) return false;
  if (!tb::wrap_shape_ok(p->dev.H, p->dev.W, p->dev.D, y_pad)) return false;
  if ((p->dev.D & 1) && !p->wrapq) return false;
  return tb::wrap_program(ops[s], alpha);
}

static int run_wrap(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad,
                    char* ws, int b0, int nb, int C, const tb_sample_ops* ops, uint32_t* minmax, hipStream_t st) {
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  tb::WrapArgs a;
  std::memset(&a, 0, sizeof(a));
  a.H = H, a.W = W, a.D = D;
  a.x = x, a.xsbc = xs[0], a.xsh = xs[1], a.xsw = xs[2];
  a.y = y, a.ysbc = ys[0], a.ysh = ys[1], a.ysw = ys[2];
  a.ypad = y_pad, a.bc0 = b0 * C, a.C = C, a.nbc = nb * C;
  a.q = p->wrapq;
  a.mm = minmax;
  a.mmp = reinterpret_cast<float2*>(ws);
  a.cnt = reinterpret_cast<uint32_t*>(ws + (size_t)tb::WRAP_MAX_WG * TB_MAX_BATCH * 8);
  // 16-B loads: contiguous rows and 16-B aligned role chunks (every row start of a 4-row chunk,
  // W/2 rows apart); 16-B stores: every output row start 16-B aligned
  const bool xal = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (xs[0] & 3) == 0 && (xs[1] & 3) == 0;
  const bool vld = (D & 1) ? (xal && xs[2] == D && (((int64_t)(W / 2) * D) & 3) == 0)
                           : (xal && (xs[2] & 3) == 0);
  const bool vst = (reinterpret_cast<uintptr_t>(y) & 15) == 0 && (ys[0] & 3) == 0 && (ys[1] & 3) == 0 && (ys[2] & 3) == 0;
  a.vec = (vld ? 1 : 0) | (vst ? 2 : 0);
  float alpha[TB_MAX_BATCH];
  for (int i = 0; i < nb; ++i) tb::wrap_program(ops[b0 + i], &alpha[i]);
  const double vox = (double)nb * C * H * W;
  Timer t(2, st, vox * (D + D + y_pad) * 4.0, (D & 1) ? "k_wrap_dgemm" : "k_wrap_even");
  TB_HIP(tb::launch_wrap(a, alpha, nb, p->ncu, st));
  return TB_OK;
}

template <int RA, int RB>
static int run_full(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad, cf* S,
                    int b0, int nb, int C, const tb_sample_ops* ops, uint32_t* minmax, hipStream_t st) {
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  const int Dh = D / 2 + 1;
  const float scale = (float)(1.0 / ((double)H * (double)W * (double)D));
  const int T = pick_tile(H, p->lds_max);
  const int ntiles = (W * Dh + T - 1) / T;
  const size_t lds_b = (size_t)tile_geo(H, T).total_cf * sizeof(cf);
  const size_t lds_s = (size_t)slab_geo(W, D).total_cf * sizeof(cf);
  BatchOps bo;
  std::memset(&bo, 0, sizeof(bo));
  for (int i = 0; i < nb; ++i) bo.s[i] = ops[b0 + i];
  // A -> B -> C per chunk of channel-volumes: a chunk's half spectrum is re-read by B and C while
  // it is still in the 256 MiB Infinity Cache (chunk_bc(); 0 = the whole group in one chain)
  const int nbc = nb * C;
  const int g = chunk_bc(p) > 0 ? chunk_bc(p) : nbc;
  for (int c0 = 0; c0 < nbc; c0 += g) {
    const int ng = (nbc - c0) < g ? (nbc - c0) : g;
    const int bc0 = b0 * C + c0;
    const double vox = (double)ng * H * W * D, spec = (double)ng * H * W * Dh * 8.0;
    const bool half = use_half(p);
    {
      Timer t(0, st, vox * 4.0 + spec, half ? "k_slab_fwd_half" : use_ct_slab(p) ? "k_slab_fwd_ct16" : "k_slab_fwd");
      if (half) {
        SlabFwdArgs a{p->dev, x, xs[0], xs[1], xs[2], S, bc0, ng};
        TB_HIP(tb::launch_slab_fwd_half(a, st));
      } else {
        const int rc = launch_slab_fwd<RA>(p, x, xs, S, bc0, ng, st);
        if (rc) return rc;
      }
    }
    {
      Timer t(1, st, 2.0 * spec,
              half ? "k_kspace_half"
              : (g_compiled_plans && p->ct_tile)
                  ? (tb::kspace_ct_persistent(W * Dh) ? "k_kspace_ct2p" : "k_kspace_ct2")
                  : "k_kspace");
      if (half) {
        KspaceArgs ka{p->dev, S, bc0, C, 32, c0, bo, ng};
        TB_HIP(tb::launch_kspace_half(ka, p->ncu, st));
      } else if (g_compiled_plans && p->ct_tile) {
        const int Tc = tb::kspace_ct_tile(W * Dh);
        KspaceArgs ka{p->dev, S, bc0, C, Tc, c0, bo, ng};
        TB_HIP(tb::launch_kspace_ct(ka, dim3((W * Dh + Tc - 1) / Tc, ng), p->ncu, st));
      } else {
        KspaceArgs ka{p->dev, S, bc0, C, T, c0, bo, ng};
        TB_HIP(launch_kspace<RB>(ka, dim3(ntiles, ng), lds_b, st));
      }
    }
    {
      Timer t(2, st, spec + (double)ng * H * W * (D + y_pad) * 4.0,
              half ? "k_slab_inv_half" : use_ct_slab(p) ? "k_slab_inv_ct" : "k_slab_inv");
      SlabInvArgs ia{p->dev, S, y, ys[0], ys[1], ys[2], y_pad, bc0, C, scale, minmax, ng};
      if (half)
        TB_HIP(tb::launch_slab_inv_half(ia, st));
      else if (use_ct_slab(p))
        TB_HIP(tb::launch_slab_inv_ct(ia, p->ncu, st));
      else
        TB_HIP(launch_slab_inv<RA>(ia, dim3(H, ng), lds_s, st));
    }
  }
  return TB_OK;
}

static int run_band(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad,
                    char* ws, int bcn_total, int b0, int nb, int C, const tb_sample_ops* ops, const BandGeo& g,
                    const BandSamplePts* sp, uint32_t* minmax, hipStream_t st) {
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  const BandWs wl = band_ws(g, H, bcn_total);
  cf* P = reinterpret_cast<cf*>(ws + wl.off_P);
  float4* AB = reinterpret_cast<float4*>(ws + wl.off_AB);
  cf* pts = reinterpret_cast<cf*>(ws + wl.off_pts);
  const int nbc = nb * C, bc0 = b0 * C;
  const double pbytes = (double)nbc * H * g.ncol * 8.0, abytes = (double)nbc * (g.KH + 1) * g.ncol * 16.0;
  tb::FwdSplit split{};
  {
    Timer t(0, st, (double)nbc * H * W * D * 4.0 + pbytes, "k_band_fwd");
    BandFwdArgs fa{p->dev, x, xs[0], xs[1], xs[2], P, bc0, nbc, g, g_band_diag & 0xff, p->tbt};
    // 16-B vector strips: contiguous rows, and 16-B aligned strips where the compiled even-D staging needs them
    const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (xs[0] & 3) == 0 && (xs[1] & 3) == 0;
    fa.vec = xs[2] == D && ((D & 1) || al || !tb::band_fwd_use_ct(D, g.NDk <= 16 ? 1 : 2));
    fa.tbt16 = p->tbt16;
    TB_HIP(tb::launch_band_fwd(fa, p->ncu, st));
    split = fa.split;
  }
  {
    Timer t(1, st, pbytes + abytes, "k_band_hcol");
    BandMidArgs ma;
    std::memset(&ma, 0, sizeof(ma));
    ma.pl = p->dev;
    ma.P = P;
    ma.AB = AB;
    ma.pts = pts;
    ma.M2F = reinterpret_cast<float*>(ws + wl.off_m2f);
    ma.scale = (float)(1.0 / ((double)H * (double)W * (double)D));
    ma.bc0 = bc0;
    ma.C = C;
    ma.cofs = 0;
    ma.nbc = nbc;
    ma.g = g;
    ma.split = split;
    int p0 = 0;
    for (int i = 0; i < nb; ++i) {
      ma.sp[i] = sp[i];
      ma.ops.s[i] = ops[b0 + i];
      ma.p0[i] = p0;
      for (int j = 0; j < sp[i].n; ++j) ma.pkd[p0 + j] = sp[i].p[j].kd;
      p0 += sp[i].n;
    }
    ma.T16 = ws + wl.off_t16;
    ma.tds = p->tds;
    ma.cnt = reinterpret_cast<uint32_t*>(ws + wl.off_cnt);
    ma.mm = g.cat ? minmax : nullptr;
    TB_HIP(tb::launch_band_mid(ma, st));
  }
  {
    // the events bracket k_band_inv16 (with the per-sample min/max keys from its last workgroup) or
    // k_band_inv alone (k_band_minmax after it runs untimed): the kernel's duration, as rocprofv3 reports it
    Timer t(2, st, abytes + (double)nbc * H * W * (D + y_pad) * 4.0, g.cat ? "k_band_inv16" : "k_band_inv");
    BandInvArgs ia;
    std::memset(&ia, 0, sizeof(ia));
    ia.pl = p->dev;
    ia.M2F = reinterpret_cast<float*>(ws + wl.off_m2f);
    ia.AB = AB;
    ia.pts = pts;
    ia.y = y;
    ia.sbc = ys[0];
    ia.sh = ys[1];
    ia.sw = ys[2];
    ia.ypad = y_pad;
    ia.bc0 = bc0;
    ia.C = C;
    ia.cofs = 0;
    ia.nbc = nbc;
    ia.scale = (float)(1.0 / ((double)H * (double)W * (double)D));
    ia.mm = minmax;
    ia.mmp = reinterpret_cast<float2*>(ws + wl.off_mmp);
    ia.tds = p->tds;
    ia.T16 = ws + wl.off_t16;
    ia.g = g;
    ia.diag = (g_band_diag >> 8) & 0xffff;
    ia.cnt = g.cat ? reinterpret_cast<uint32_t*>(ws + wl.off_cnt) : nullptr;
    for (int i = 0; i < nb; ++i) ia.sp[i] = sp[i];
    TB_HIP(tb::launch_band_inv(ia, p->ncu, st));
  }
  // the split-f16 C' writes the keys from its last workgroup; the f32 C' leaves them to k_band_minmax
  if (minmax && !g.cat) TB_HIP(tb::launch_band_minmax(reinterpret_cast<float2*>(ws + wl.off_mmp), minmax, b0 * C, C, nbc, H, W, st));
  return TB_OK;
}

// full-spectrum route of a plan the mixed-radix passes do not take (tb_plan::generic)
static int run_generic(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad,
                       void* ws, int b0, int nb, int C, const tb_sample_ops* ops, uint32_t* minmax, hipStream_t st) {
  BatchOps bo;
  std::memset(&bo, 0, sizeof(bo));
  for (int i = 0; i < nb; ++i) bo.s[i] = ops[b0 + i];
  const double vox = (double)nb * C * p->dev.H * p->dev.W * p->dev.D;
  Timer t(1, st, vox * (4.0 + 2.0 * 16.0 * 6.0 + 16.0 + 4.0), "k_gen_dft");
  const GenLaunch g{p->dev, x, xs, y, ys, static_cast<cf*>(ws), y_pad, b0 * C, C, nb * C, minmax, &bo};
  TB_HIP(tb::launch_gen_filter(g, st));
  return TB_OK;
}

// Samples per chain of the closed-form route's three launches (0 = the whole launch group): per-sample chains would let k_point_apply re-read a 142 MB sample from the Infinity
// Cache, but cost more in launches and smaller grids than they saved.
static int point_chunk(const tb_plan* p, int C) {
  (void)p;
  (void)C;
  return 0;  // measured: one sample per chain 0.240 vs 0.213 ms per C3 step (planes)
}

static int run_point(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad,
                     char* ws, int b0, int nb, int C, const tb_sample_ops* ops, uint32_t* minmax,
                     hipStream_t st) {
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  const int cs = point_chunk(p, C) > 0 ? point_chunk(p, C) : nb;
  for (int s0 = 0; s0 < nb; s0 += cs) {
    const int ns = nb - s0 < cs ? nb - s0 : cs, sb = b0 + s0;
    const int nbc = ns * C;
    tb::PointArgs a;
    std::memset(&a, 0, sizeof(a));
    a.H = H, a.W = W, a.D = D;
    a.x = x, a.xsbc = xs[0], a.xsh = xs[1], a.xsw = xs[2];
    a.y = y, a.ysbc = ys[0], a.ysh = ys[1], a.ysw = ys[2];
    a.ypad = y_pad, a.bc0 = sb * C, a.C = C, a.nbc = nbc, a.mm = minmax;
    const tb::PointWs wl = tb::point_ws(nbc);
    a.part = reinterpret_cast<double*>(ws + wl.part);
    a.delta = reinterpret_cast<float*>(ws + wl.delta);
    a.mmp = reinterpret_cast<float2*>(ws + wl.mmp);
    a.cnt = reinterpret_cast<uint32_t*>(ws + wl.cnt);
    a.namax = 1;
    for (int i = 0; i < ns; ++i) {
      a.ops.s[i] = ops[sb + i];
      for (int c = 0; c < C; ++c) {
        int n = 0;
        for (int o = 0; o < ops[sb + i].n; ++o) n += ops[sb + i].op[o].chan < 0 || ops[sb + i].op[o].chan == c;
        a.namax = n > a.namax ? n : a.namax;
      }
    }
    tb::point_grid(a, p->ncu);
    const double vox = (double)nbc * H * W * D;
    {
      Timer t(0, st, vox * 4.0, "k_point_dft");
      TB_HIP(tb::launch_point(a, st, 0));
    }
    {
      Timer t(1, st, (double)nbc * a.parts * TB_MAX_OPS * 16.0, "k_point_delta");
      TB_HIP(tb::launch_point(a, st, 1));
    }
    {
      Timer t(2, st, vox * 4.0 + (double)nbc * H * W * (D + y_pad) * 4.0, "k_point_apply");
      TB_HIP(tb::launch_point(a, st, 2));
    }
  }
  return TB_OK;
}

static int run_copy(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad, int b0,
                    int nb, int C, uint32_t* minmax, hipStream_t st) {
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  const int nbc = nb * C;
  Timer t(2, st, (double)nbc * H * W * (2.0 * D + y_pad) * 4.0, "k_copy_pad");
  CopyArgs ca{x, xs[0], xs[1], xs[2], y, ys[0], ys[1], ys[2], H, W, D, y_pad, b0 * C, C, nbc, minmax};
  TB_HIP(tb::launch_copy_pad(ca, st));
  return TB_OK;
}

template <int RA, int RB>
static int kspace_filter(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad,
                         void* ws, size_t ws_bytes, int B, int C, const tb_sample_ops* ops, uint32_t* minmax,
                         void* stream) {
  if (!p || !x || !y || !xs || !ys || !ops || B < 1 || C < 1 || y_pad < 0) return TB_ERR_INVALID_ARG;
  if (ws_bytes < tb_workspace_bytes(p, B * C) || !ws) return TB_ERR_WORKSPACE;
  for (int b = 0; b < B; ++b)
    if (ops[b].n < 0 || ops[b].n > TB_MAX_OPS) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // Runs of consecutive samples with the same route, in launch groups of <= TB_MAX_BATCH samples
  // (the op programs travel in the kernel arguments): empty programs are copied through (the
  // reference returns the input untouched), low-pass programs take the band passes A'/B'/C',
  // the rest the full-spectrum passes A/B/C.  Routes are planned first: the band passes write
  // their samples' min/max keys outright, the others accumulate them atomically from a reset.
  struct Run {
    int s0, s1, route;
    BandGeo g;
    BandSamplePts sp[TB_MAX_BATCH];
  };
  std::vector<Run> runs;
  bool atomic_keys = false;
  for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
    const int nb = (B - b0) < TB_MAX_BATCH ? (B - b0) : TB_MAX_BATCH;
    int i = 0;
    while (i < nb) {
      float al0 = 0.f, al = 0.f;
      auto route = [&](int s, float* alpha) {
        return ops[s].n == 0 ? RUN_COPY : (wrap_run(p, ops, s, y_pad, ws_bytes, alpha) ? RUN_WRAP : RUN_FULL);
      };
      Run run;
      run.route = route(b0 + i, &al0);
      int j = i + 1;
      // odd D: one circulant table per launch (k_wrap_dgemm builds it from one alpha); even D: k_wrap_even
      // carries every sample's 2-tap weights, so mixed alphas share the launch
      while (j < nb && route(b0 + j, &al) == run.route && (run.route != RUN_WRAP || al == al0 || !(p->dev.D & 1))) ++j;
      run.s0 = b0 + i;
      run.s1 = b0 + j;
      if (run.route == RUN_FULL && g_point && ws_bytes >= tb::point_ws(B * C).total &&
          tb::point_strides_ok(p->dev.H, p->dev.W, p->dev.D, y_pad, xs, ys)) {
        bool pt = true;
        for (int s = run.s0; s < run.s1 && pt; ++s) pt = tb::point_program(ops[s], p->dev.H, p->dev.W, p->dev.D);
        if (pt) run.route = RUN_POINT;
      }
      if (run.route == RUN_FULL && g_band && band_plan(p, ops, run.s0, run.s1, y_pad, ws_bytes, B * C, run.g, run.sp))
        run.route = RUN_BAND;
      atomic_keys |= run.route == RUN_COPY || run.route == RUN_FULL;  // the other routes write their keys outright
      runs.push_back(run);
      i = j;
    }
  }
  if (minmax && atomic_keys) {
    hipLaunchKernelGGL(k_minmax_init, dim3((B + 255) / 256), dim3(256), 0, st, minmax, B);
    TB_HIP(hipGetLastError());
  }
  for (const Run& run : runs) {
    const int nb = run.s1 - run.s0;
    int rc = TB_OK;
    if (run.route == RUN_COPY)
      rc = run_copy(p, x, xs, y, ys, y_pad, run.s0, nb, C, minmax, st);
    else if (run.route == RUN_WRAP)
      rc = run_wrap(p, x, xs, y, ys, y_pad, static_cast<char*>(ws), run.s0, nb, C, ops, minmax, st);
    else if (run.route == RUN_POINT)
      rc = run_point(p, x, xs, y, ys, y_pad, static_cast<char*>(ws), run.s0, nb, C, ops, minmax, st);
    else if (run.route == RUN_BAND)
      rc = run_band(p, x, xs, y, ys, y_pad, static_cast<char*>(ws), B * C, run.s0, nb, C, ops, run.g, run.sp, minmax,
                    st);
    else if (p->generic)
      rc = run_generic(p, x, xs, y, ys, y_pad, ws, run.s0, nb, C, ops, minmax, st);
    else
      rc = run_full<RA, RB>(p, x, xs, y, ys, y_pad, static_cast<cf*>(ws), run.s0, nb, C, ops, minmax, st);
    if (rc) return rc;
  }
  return TB_OK;
}

template <int RA, int RB>
static int kspace_stats(const tb_plan* p, const float* x, const int64_t* xs, void* ws, size_t ws_bytes, int B,
                             int C, const tb_sample_ops* ops, double* out, void* stream) {
  if (!p || !x || !xs || !ops || !out || B < 1 || C < 1) return TB_ERR_INVALID_ARG;
  if (ws_bytes < tb_workspace_bytes(p, B * C) || !ws) return TB_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  cf* S = static_cast<cf*>(ws);
  const int H = p->dev.H, W = p->dev.W, D = p->dev.D;
  const int T = pick_tile(H, p->lds_max);
  const int ntiles = (W * (D / 2 + 1) + T - 1) / T;
  const size_t lds_b = (size_t)tile_geo(H, T).total_cf * sizeof(cf);
  int rc = TB_OK;
  TB_HIP(hipMemsetAsync(out, 0, sizeof(double) * B * C, st));
  if (p->generic) {
    for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
      const int nb = (B - b0) < TB_MAX_BATCH ? (B - b0) : TB_MAX_BATCH;
      BatchOps bo;
      std::memset(&bo, 0, sizeof(bo));
      for (int i = 0; i < nb; ++i) bo.s[i] = ops[b0 + i];
      const GenLaunch g{p->dev, x, xs, nullptr, nullptr, S, 0, b0 * C, C, nb * C, nullptr, &bo};
      TB_HIP(tb::launch_gen_logabs(g, out, st));
    }
    return TB_OK;
  }
  for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
    const int nb = (B - b0) < TB_MAX_BATCH ? (B - b0) : TB_MAX_BATCH;
    BatchOps bo;
    std::memset(&bo, 0, sizeof(bo));
    for (int i = 0; i < nb; ++i) bo.s[i] = ops[b0 + i];
    rc = launch_slab_fwd<RA>(p, x, xs, S, b0 * C, nb * C, st);
    if (rc) return rc;
    StatsArgs sa{p->dev, S, b0 * C, C, T, 0, out, bo};
    TB_HIP(launch_kspace_stats<RB>(sa, dim3(ntiles, nb * C), lds_b, st));
  }
  return TB_OK;
}

int tb_kspace_filter_f32(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys, int y_pad,
                         void* ws, size_t ws_bytes, int B, int C, const tb_sample_ops* ops, uint32_t* minmax,
                         void* stream) {
  if (!p) return TB_ERR_INVALID_ARG;
#define TB_ARGS p, x, xs, y, ys, y_pad, ws, ws_bytes, B, C, ops, minmax, stream
  if (p->rset_wd == RS_SMALL)
    return p->rset_h == RS_SMALL ? kspace_filter<RS_SMALL, RS_SMALL>(TB_ARGS) : kspace_filter<RS_SMALL, RS_ALL>(TB_ARGS);
  return p->rset_h == RS_SMALL ? kspace_filter<RS_ALL, RS_SMALL>(TB_ARGS) : kspace_filter<RS_ALL, RS_ALL>(TB_ARGS);
#undef TB_ARGS
}

int tb_planes_closed_form_f32(const tb_plan* p, const float* x, const int64_t* xs, float* y, const int64_t* ys,
                              int y_pad, void* ws, size_t ws_bytes, int B, int C, const tb_sample_ops* ops,
                              uint32_t* minmax, void* stream) {
  if (!p || !x || !y || !xs || !ys || !ops || B < 1 || C < 1 || y_pad < 0 || !ws) return TB_ERR_INVALID_ARG;
  if (ws_bytes < tb::point_ws(B * C).total) return TB_ERR_WORKSPACE;
  for (int b = 0; b < B; ++b)
    if (ops[b].n < 1 || ops[b].n > TB_MAX_OPS || !tb::point_program(ops[b], p->dev.H, p->dev.W, p->dev.D))
      return TB_ERR_INVALID_ARG;  // not spike-only, or two spikes touch: tb_kspace_filter_f32 takes those
  if (!tb::point_strides_ok(p->dev.H, p->dev.W, p->dev.D, y_pad, xs, ys)) return TB_ERR_UNSUPPORTED_SIZE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
    const int nb = (B - b0) < TB_MAX_BATCH ? (B - b0) : TB_MAX_BATCH;
    const int rc = run_point(p, x, xs, y, ys, y_pad, static_cast<char*>(ws), b0, nb, C, ops, minmax, st);
    if (rc) return rc;
  }
  return TB_OK;
}

int tb_kspace_logabs_sum_f32(const tb_plan* p, const float* x, const int64_t* xs, void* ws, size_t ws_bytes, int B,
                             int C, const tb_sample_ops* ops, double* out, void* stream) {
  if (!p) return TB_ERR_INVALID_ARG;
#define TB_ARGS p, x, xs, ws, ws_bytes, B, C, ops, out, stream
  if (p->rset_wd == RS_SMALL)
    return p->rset_h == RS_SMALL ? kspace_stats<RS_SMALL, RS_SMALL>(TB_ARGS) : kspace_stats<RS_SMALL, RS_ALL>(TB_ARGS);
  return p->rset_h == RS_SMALL ? kspace_stats<RS_ALL, RS_SMALL>(TB_ARGS) : kspace_stats<RS_ALL, RS_ALL>(TB_ARGS);
#undef TB_ARGS
}

int tb_minmax_f32(const float* x, uint32_t* mm, int B, int64_t rows, int len, int64_t ld, int64_t sb, void* stream) {
  if (!x || !mm || B < 1 || rows < 1 || len < 1 || ld < len) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  Timer t(3, st, (double)B * rows * len * 4.0, "k_minmax");
  hipLaunchKernelGGL(k_minmax_init, dim3((B + 255) / 256), dim3(256), 0, st, mm, B);
  const int64_t n = rows * len;
  int64_t blocks = (n + 256 * 8 - 1) / (256 * 8);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_minmax<256>, dim3((unsigned)blocks, B), dim3(256), 0, st, x, mm, rows, len, ld, sb);
  TB_HIP(hipGetLastError());
  return TB_OK;
}

int tb_salt_pepper_f32(const float* x, float* y, int8_t* cls, const float* u_in, uint64_t seed, uint64_t offset,
                       const float* thr, const uint32_t* mm, int B, int64_t rows, int len, int64_t ld, int64_t sb,
                       void* stream) {
  if (!x || !y || !thr || !mm || B < 1 || rows < 1 || len < 1 || ld < len) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = rows * len;
  if (u_in) {  // parity mode: the caller's uniform field, one class per voxel
    int64_t blocks = ((n + 3) / 4 + NT_SAP - 1) / NT_SAP;
    if (blocks > 2048) blocks = 2048;
    Timer t(3, st, (double)B * n * (12.0 + (cls ? 1.0 : 0.0)), "k_salt_pepper");
    for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
      const int nb = (B - b0) < TB_MAX_BATCH ? (B - b0) : TB_MAX_BATCH;
      SapThr th;
      for (int i = 0; i < TB_MAX_BATCH; ++i) {
        th.lo[i] = i < nb ? thr[2 * (b0 + i)] : 0.f;
        th.hi[i] = i < nb ? thr[2 * (b0 + i) + 1] : 0.f;
      }
      hipLaunchKernelGGL(k_salt_pepper<NT_SAP>, dim3((unsigned)blocks, nb), dim3(NT_SAP), 0, st, x, y, cls, u_in, seed,
                         offset, th, mm, b0, rows, len, ld, sb, 0);
      TB_HIP(hipGetLastError());
    }
    return TB_OK;
  }
  // device stream: out of place = copy, then the sparse scatter of the changed voxels (the class
  // map, when asked for, is zeroed first); in place only the changed voxels are written
  for (int b = 0; b < B; ++b) {
    if (x != y)
      TB_HIP(hipMemcpy2DAsync(y + b * sb, ld * 4, x + b * sb, ld * 4, (size_t)len * 4, rows, hipMemcpyDeviceToDevice, st));
    if (cls) TB_HIP(hipMemset2DAsync(cls + b * sb, ld, 0, (size_t)len, rows, st));
  }
  // algorithmic bytes: one 4-B store per changed voxel (~p n), no reads
  double changed = 0.0;
  for (int b = 0; b < B; ++b) changed += (double)n * (thr[2 * b + 1] > 0.f ? (thr[2 * b + 1] < 1.f ? thr[2 * b + 1] : 1.f) : 0.f);
  Timer t(3, st, changed * (4.0 + (cls ? 1.0 : 0.0)), "k_sap_geom");
  const int64_t segs = (n + SAP_SEG - 1) / SAP_SEG;
  for (int b0 = 0; b0 < B; b0 += TB_MAX_BATCH) {
    const int nb = (B - b0) < TB_MAX_BATCH ? (B - b0) : TB_MAX_BATCH;
    SapGeomArgs ga;
    ga.y = y;
    ga.cls = cls;
    ga.seed = seed;
    ga.offset = offset;
    for (int i = 0; i < TB_MAX_BATCH; ++i) {
      ga.lo[i] = i < nb ? thr[2 * (b0 + i)] : 0.f;
      ga.hi[i] = i < nb ? thr[2 * (b0 + i) + 1] : 0.f;
    }
    ga.mm = mm;
    ga.b0 = b0;
    ga.rows = rows;
    ga.len = len;
    ga.ld = ld;
    ga.sb = sb;
    hipLaunchKernelGGL(k_sap_geom, dim3((unsigned)((segs + 255) / 256), nb), dim3(256), 0, st, ga);
    TB_HIP(hipGetLastError());
  }
  return TB_OK;
}

float tb_key_to_float(uint32_t key) { return key2f(key); }

int tb_disk_mask_f32(float* mask, int64_t outer, int n0, int n1, int n2, int int_r, int64_t r2i, float r2f,
                     int inside_off, void* stream) {
  if (!mask || outer < 1 || n0 < 1 || n1 < 1 || n2 < 1) return TB_ERR_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = outer * n0 * n1 * n2;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_disk_mask, dim3((unsigned)blocks), dim3(256), 0, st, mask, outer, n0, n1, n2, int_r, r2i, r2f,
                     inside_off);
  TB_HIP(hipGetLastError());
  return TB_OK;
}

int tb_set_chain_chunk(int n) {
  g_chunk = n;
  return TB_OK;
}

int tb_set_compiled_plans(int enable) {
  g_compiled_plans = enable != 0;
  return TB_OK;
}

int tb_set_band_plans(int enable) {
  g_band = enable != 0;
  return TB_OK;
}

int tb_set_wrap_plans(int enable) {
  g_wrap = enable != 0;
  return TB_OK;
}

int tb_set_half_units(int enable) {
  g_half = enable != 0;
  return TB_OK;
}

int tb_set_point_plans(int enable) {
  g_point = enable != 0;
  return TB_OK;
}

int tb_set_band_inv16(int enable) {
  g_inv16 = enable != 0;
  return TB_OK;
}

int tb_set_pass_timing(int enable) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_timing = enable != 0;
  for (auto& r : g_recs) { g_pool.push_back(r.a); g_pool.push_back(r.b); }
  g_recs.clear();
  return TB_OK;
}

int tb_get_pass_stats(float* ms, int* cnt, double* bytes) {
  if (!ms || !cnt) return TB_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_tmu);
  for (int i = 0; i < 4; ++i) {
    ms[i] = 0.f;
    cnt[i] = 0;
    if (bytes) bytes[i] = 0.0;
  }
  for (auto& r : g_recs) {
    TB_HIP(hipEventSynchronize(r.b));
    float t = 0.f;
    TB_HIP(hipEventElapsedTime(&t, r.a, r.b));
    ms[r.slot] += t;
    cnt[r.slot] += 1;
    if (bytes) bytes[r.slot] += r.bytes;
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_recs.clear();
  return TB_OK;
}

int tb_get_pass_times_ms(float* ms, int* cnt) { return tb_get_pass_stats(ms, cnt, nullptr); }

const char* tb_pass_kernel(int slot) {
  if (slot < 0 || slot > 3) return "";
  std::lock_guard<std::mutex> lk(g_tmu);
  return g_slot_kernel[slot];
}
