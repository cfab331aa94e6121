// Streaming-read ceiling microbenchmark (not part of the library): how fast can one kernel read a
// C3-sized f32 array (2 x 4 x 240 x 240 x 155 = 285.7 MB) on this GPU, and what does a preceding
// large write cost the read (the dirty-line write-back measured by scripts/diag/mall.py)?
// Variants: grid (persistent k x CUs or one pass), threads per workgroup, float4 loads per thread
// per iteration, nontemporal loads.  Prints one JSON line per variant (best and mean of the reps).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

template <int UNR, bool NT>
__global__ void k_read(const f4* __restrict__ x, long n4, float* __restrict__ out) {
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNR - 1) * stride < n4; i += UNR * stride) {
    f4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u * stride) : x[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u];
  }
  for (; i < n4; i += stride) acc += x[i];
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == -1.2345f) out[threadIdx.x] = s;  // keeps the loads live
}

__global__ void k_fill(f4* y, long n4, float v) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    y[i] = f4{v, v, v, v};
}

__global__ void k_fill_nt(f4* y, long n4, float v) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(f4{v, v, v, v}, y + i);
}

__global__ void k_copy_nt(const f4* __restrict__ x, f4* __restrict__ y, long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(x + i), y + i);
}

__global__ void k_copy(const f4* __restrict__ x, f4* __restrict__ y, long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) y[i] = x[i];
}

struct Res {
  float best, mean;
};

template <class F>
static Res timeit(F launch, int dirty, f4* junk, long nj4, int ncu, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    if (dirty == 1) k_fill<<<ncu * 8, 256>>>(junk, nj4, (float)r);
    if (dirty == 2) k_fill_nt<<<ncu * 8, 256>>>(junk, nj4, (float)r);
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
  const long n = argc > 1 ? std::atol(argv[1]) : 2L * 4 * 240 * 240 * 155;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const long n4 = n / 4, nj4 = (long)(294e6 / 16);
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int ncu = pr.multiProcessorCount;
  f4 *x, *junk, *y;
  float* out;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&y, n4 * 16));
  CK(hipMalloc(&junk, nj4 * 16));
  CK(hipMalloc(&out, 4096));
  k_fill<<<ncu * 8, 256>>>(x, n4, 1.f);
  CK(hipDeviceSynchronize());
  const double bytes = (double)n4 * 16;
  auto report = [&](const char* name, int grid, int nt, Res r, int dirty, double by) {
    std::printf("{\"kernel\": \"%s\", \"grid\": %d, \"threads\": %d, \"after\": \"%s\", \"best_us\": %.1f, "
                "\"mean_us\": %.1f, \"best_TBs\": %.3f, \"mean_TBs\": %.3f}\n",
                name, grid, nt, dirty == 2 ? "nt_write" : (dirty ? "write" : "read"), r.best, r.mean, by / r.best / 1e6, by / r.mean / 1e6);
    std::fflush(stdout);
  };
#define RUN(UNR, NTL, NT, GRID, NAME)                                                                    \
  for (int dirty = 0; dirty < 2; ++dirty) {                                                             \
    const int g = (GRID);                                                                               \
    Res r = timeit([&] { k_read<UNR, NTL><<<g, NT>>>(x, n4, out); }, dirty, junk, nj4, ncu, reps);       \
    report(NAME, g, NT, r, dirty, bytes);                                                               \
  }
  const long one_pass256 = (n4 + 255) / 256, one_pass_u4 = (n4 / 4 + 255) / 256;
  RUN(1, false, 256, (int)one_pass256, "read_u1_onepass");
  RUN(4, false, 256, (int)one_pass_u4, "read_u4_onepass");
  for (int k : {4, 8, 16, 32}) {
    RUN(4, false, 256, ncu * k, "read_u4");
    RUN(8, false, 256, ncu * k, "read_u8");
  }
  for (int k : {2, 4, 8}) {
    RUN(4, false, 512, ncu * k, "read_u4");
    RUN(4, false, 1024, ncu * k, "read_u4");
    RUN(4, true, 512, ncu * k, "read_u4_nt");
  }
  for (int dirty = 0; dirty < 3; ++dirty) {
    Res r = timeit([&] { k_copy<<<ncu * 16, 256>>>(x, y, n4); }, dirty, junk, nj4, ncu, reps);
    report("copy", ncu * 16, 256, r, dirty, 2 * bytes);
    r = timeit([&] { k_copy_nt<<<ncu * 16, 256>>>(x, y, n4); }, dirty, junk, nj4, ncu, reps);
    report("copy_nt", ncu * 16, 256, r, dirty, 2 * bytes);
    Res w = timeit([&] { k_fill<<<ncu * 16, 256>>>(y, n4, 2.f); }, dirty, junk, nj4, ncu, reps);
    report("fill", ncu * 16, 256, w, dirty, bytes);
    w = timeit([&] { k_fill_nt<<<ncu * 16, 256>>>(y, n4, 2.f); }, dirty, junk, nj4, ncu, reps);
    report("fill_nt", ncu * 16, 256, w, dirty, bytes);
    r = timeit([&] { k_read<4, false><<<ncu * 4, 1024>>>(x, n4, out); }, dirty, junk, nj4, ncu, reps);
    report("read_u4", ncu * 4, 1024, r, dirty, bytes);
    r = timeit([&] { k_read<4, true><<<ncu * 4, 1024>>>(x, n4, out); }, dirty, junk, nj4, ncu, reps);
    report("read_u4_nt", ncu * 4, 1024, r, dirty, bytes);
  }
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(junk));
  CK(hipFree(out));
  return 0;
}
