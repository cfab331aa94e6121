// Access-order microbenchmark for the band passes (not part of the library).
//
// Pass A' reads its 285.7 MB as 16-row strips (9,920 B) with each persistent wave owning a
// contiguous range of strips; pass C' writes 20 KB units (32 rows x 640 B) with each workgroup
// owning a contiguous range of units.  At any moment the waves then touch addresses spread over the
// whole array.  This measures the same access shapes in grid-stride order (the concurrently touched
// addresses form one compact window), with and without a compute gap per strip / unit, and the two
// kinds of timing events (default = system-scope fences, hipEventDisableSystemFence).
//   hipcc --offload-arch=gfx950 -O3 order_bw.hip -o order_bw && ./order_bw [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

constexpr int STRIP_Q = 620;  // 16-B vectors per strip (16 rows x 155 floats)
constexpr int PF = 10;        // per lane

// ORDER 0: wave gw owns strips [gw * NS / G, (gw + 1) * NS / G); 1: strips gw, gw + G, ...
template <int ORDER, int SLEEP>
__global__ __launch_bounds__(256) void k_strip_read(const f4* __restrict__ x, int ns, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int G = gridDim.x * 4, gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  int t, t1, step;
  if (ORDER == 0) {
    t = (int)((long)gw * ns / G);
    t1 = (int)((long)(gw + 1) * ns / G);
    step = 1;
  } else {
    t = gw;
    t1 = ns;
    step = G;
  }
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  f4 pf[PF];
  auto load = [&](int s) {
    const f4* p = x + (long)s * STRIP_Q;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int q = lane + 64 * u;
      if (q < STRIP_Q) pf[u] = __builtin_nontemporal_load(p + q);
    }
  };
  if (t < t1) load(t);
  while (t < t1) {
    f4 cur[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) cur[u] = pf[u];
    const int tn = t + step;
    if (tn < t1) load(tn);
#pragma unroll
    for (int u = 0; u < PF; ++u) acc += cur[u];
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    t = tn;
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == -1.2345f) out[threadIdx.x] = s;
}

constexpr int UNIT_F = 32 * 160;  // floats per C' unit (32 rows x 160 columns)

// 16-wave workgroups.  ORDER 0: workgroup b owns units [b * per, (b + 1) * per), wave w takes every
// 16th of them; 1: unit u = global wave + k * (waves in the grid).  Per unit 5 column tiles x 4
// stores, each instruction 8 whole 128-B rows (row stride 640 B), as pass C' after tile_rows8.
template <int ORDER, int SLEEP>
__global__ __launch_bounds__(1024) void k_unit_write(f4* __restrict__ y, int nu, float v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int u, ue, step;
  if (ORDER == 0) {
    const int per = (nu + gridDim.x - 1) / gridDim.x;
    const int ub = blockIdx.x * per;
    u = ub + wv;
    ue = std::min(ub + per, nu);
    step = 16;
  } else {
    u = blockIdx.x * 16 + wv;
    ue = nu;
    step = gridDim.x * 16;
  }
  const int r = lane & 7, c = lane >> 3;
  for (; u < ue; u += step) {
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    float* base = reinterpret_cast<float*>(y) + (long)u * UNIT_F;
    for (int nt = 0; nt < 5; ++nt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f4* dst = reinterpret_cast<f4*>(base + (8 * k + r) * 160 + 32 * nt + 4 * c);
        *dst = f4{v, v + k, v + nt, v};
      }
  }
}

__global__ void k_fill(f4* y, long n4, float v) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    y[i] = f4{v, v, v, v};
}

struct Res {
  float best, mean;
};

template <class F>
static Res timeit(F launch, bool nofence, bool dirty, f4* junk, long nj4, int ncu, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreateWithFlags(&a, nofence ? hipEventDisableSystemFence : 0));
  CK(hipEventCreateWithFlags(&b, nofence ? hipEventDisableSystemFence : 0));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    if (dirty) k_fill<<<ncu * 8, 256>>>(junk, nj4, (float)r);
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) t.push_back(ms * 1e3f);
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  float s = 0;
  for (float v : t) s += v;
  return {*std::min_element(t.begin(), t.end()), s / t.size()};
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const int ns = 28800;                 // C3 strips: 8 channel-volumes x 240 slabs x 15 strips
  const int nu = 15360;                 // C3 units: 1920 slabs x 8 row tiles
  const long nx4 = (long)ns * STRIP_Q;  // 285.7 MB
  const long ny4 = (long)nu * UNIT_F / 4;
  const long nj4 = (long)(294e6 / 16);
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int ncu = pr.multiProcessorCount;
  f4 *x, *y, *junk;
  float* out;
  CK(hipMalloc(&x, nx4 * 16));
  CK(hipMalloc(&y, ny4 * 16));
  CK(hipMalloc(&junk, nj4 * 16));
  CK(hipMalloc(&out, 4096));
  k_fill<<<ncu * 8, 256>>>(x, nx4, 1.f);
  CK(hipDeviceSynchronize());
  auto report = [&](const char* name, bool nofence, bool dirty, Res r, double by) {
    std::printf("{\"kernel\": \"%s\", \"events\": \"%s\", \"after\": \"%s\", \"best_us\": %.2f, \"mean_us\": %.2f, "
                "\"best_TBs\": %.3f, \"mean_TBs\": %.3f}\n",
                name, nofence ? "no_fence" : "default", dirty ? "write" : "idle", r.best, r.mean, by / r.best / 1e6,
                by / r.mean / 1e6);
    std::fflush(stdout);
  };
  const double rb = (double)nx4 * 16, wb = (double)ny4 * 16;
  for (int nf = 0; nf < 2; ++nf)
    for (int dirty = 0; dirty < 2; ++dirty) {
      const int g = ncu * 3;  // 3 four-wave blocks per CU (pass A''s occupancy)
      report("strip_read_ranges", nf, dirty, timeit([&] { k_strip_read<0, 0><<<g, 256>>>(x, ns, out); }, nf, dirty, junk, nj4, ncu, reps), rb);
      report("strip_read_stride", nf, dirty, timeit([&] { k_strip_read<1, 0><<<g, 256>>>(x, ns, out); }, nf, dirty, junk, nj4, ncu, reps), rb);
      report("strip_read_ranges_sleep", nf, dirty, timeit([&] { k_strip_read<0, 24><<<g, 256>>>(x, ns, out); }, nf, dirty, junk, nj4, ncu, reps), rb);
      report("strip_read_stride_sleep", nf, dirty, timeit([&] { k_strip_read<1, 24><<<g, 256>>>(x, ns, out); }, nf, dirty, junk, nj4, ncu, reps), rb);
      report("unit_write_ranges", nf, dirty, timeit([&] { k_unit_write<0, 0><<<ncu, 1024>>>(y, nu, 2.f); }, nf, dirty, junk, nj4, ncu, reps), wb);
      report("unit_write_stride", nf, dirty, timeit([&] { k_unit_write<1, 0><<<ncu, 1024>>>(y, nu, 2.f); }, nf, dirty, junk, nj4, ncu, reps), wb);
      report("unit_write_ranges_sleep", nf, dirty, timeit([&] { k_unit_write<0, 12><<<ncu, 1024>>>(y, nu, 2.f); }, nf, dirty, junk, nj4, ncu, reps), wb);
      report("unit_write_stride_sleep", nf, dirty, timeit([&] { k_unit_write<1, 12><<<ncu, 1024>>>(y, nu, 2.f); }, nf, dirty, junk, nj4, ncu, reps), wb);
      report("fill", nf, dirty, timeit([&] { k_fill<<<ncu * 16, 256>>>(y, ny4, 3.f); }, nf, dirty, junk, nj4, ncu, reps), wb);
    }
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(junk));
  CK(hipFree(out));
  return 0;
}
