// Store-pattern microbenchmark for pass C' (not part of the library): writes a
// [units][32 rows][160] f32 array (units = 1920 slabs x 8 tiles, 295 MB) with different
// per-instruction footprints, persistent grids of G workgroups x 256 threads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int ROWP = 160, TR = 32;
constexpr long UNITS = 1920L * 8;

// P0: linear grid-stride fill of the whole array
__global__ void p_linear(f32x4* y, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) y[i] = f32x4{1.f, 2.f, 3.f, 4.f};
}
// P1: unit per wave; per instruction 8 rows x 128 B (lane>>3 row, lane&7 16-B piece), 5 column chunks
__global__ void p_rowseg(float* y, int mode) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c4 = lane & 7;
  for (long u = blockIdx.x * 4L + wv; u < UNITS; u += gridDim.x * 4L) {
    float* t = y + u * TR * ROWP;
    if (mode == 0) {  // row segments, chunk-major (our C': all rows of chunk 0, then chunk 1, ...)
      for (int ch = 0; ch < 5; ++ch)
        for (int k = 0; k < 4; ++k) {
          const int r = (lane >> 3) + 8 * k;
          *reinterpret_cast<f32x4*>(t + r * ROWP + ch * 32 + 4 * c4) = f32x4{1.f, 2.f, 3.f, 4.f};
        }
    } else if (mode == 1) {  // contiguous 1 KB per instruction
      for (int i = 0; i < TR * ROWP / 256; ++i)
        *reinterpret_cast<f32x4*>(t + i * 256 + 4 * lane) = f32x4{1.f, 2.f, 3.f, 4.f};
    } else {  // row segments, misaligned by 1 float for the upper half (mirror-like: starts at col 124)
      for (int ch = 0; ch < 5; ++ch)
        for (int k = 0; k < 4; ++k) {
          const int r = (lane >> 3) + 8 * k;
          const int c = ch < 2 ? ch * 32 + 4 * c4 : 60 + (ch - 2) * 32 + 4 * c4;  // 2 aligned, 3 shifted chunks
          if (c + 4 <= ROWP) *reinterpret_cast<f32x4*>(t + r * ROWP + c) = f32x4{1.f, 2.f, 3.f, 4.f};
        }
    }
  }
}
// P2: per lane one row, 16 B per lane at column 8g+4hl (MFMA accumulator layout, no staging)
__global__ void p_lanerow(float* y) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l31 = lane & 31, hl = lane >> 5;
  for (long u = blockIdx.x * 4L + wv; u < UNITS; u += gridDim.x * 4L) {
    float* t = y + u * TR * ROWP + l31 * ROWP;
    for (int nt = 0; nt < 5; ++nt)
      for (int g = 0; g < 4; ++g) *reinterpret_cast<f32x4*>(t + nt * 32 + 8 * g + 4 * hl) = f32x4{1.f, 2.f, 3.f, 4.f};
  }
}

// P3: MFMA-layout values staged through LDS per half-tile (as pass C'), then row-segment stores
__global__ __launch_bounds__(256) void p_staged(float* y, int nhalf) {
  __shared__ __attribute__((aligned(16))) float stg_all[4][32 * 36];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l31 = lane & 31, hl = lane >> 5, c4 = lane & 7;
  float* stg = stg_all[wv];
  for (long u = blockIdx.x * 4L + wv; u < UNITS; u += gridDim.x * 4L) {
    float* t = y + u * TR * ROWP;
    for (int h = 0; h < nhalf; ++h) {
      const int ch = h % 5;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(stg + l31 * 36 + 8 * g + 4 * hl) = f32x4{(float)g, 1.f, 2.f, (float)h};
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = (lane >> 3) + 8 * k;
        *reinterpret_cast<f32x4*>(t + r * ROWP + ch * 32 + 4 * c4) = *reinterpret_cast<const f32x4*>(stg + r * 36 + 4 * c4);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

int main() {
  const long n = UNITS * TR * ROWP;
  float* y;
  hipMalloc(&y, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    printf("%-34s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, n * 4 / (ms * 1e-3) / 1e9);
  };
  run("linear fill 4096x256", [&] { p_linear<<<4096, 256>>>((f32x4*)y, n / 4); });
  run("linear fill 1024x256", [&] { p_linear<<<1024, 256>>>((f32x4*)y, n / 4); });
  run("staged 5 halves G=768", [&] { p_staged<<<768, 256>>>(y, 5); });
  run("staged 6 halves G=768", [&] { p_staged<<<768, 256>>>(y, 6); });
  run("staged 5 halves G=1024", [&] { p_staged<<<1024, 256>>>(y, 5); });
  for (int g : {768, 1024}) {
    char b[64];
    snprintf(b, 64, "rowseg chunk-major G=%d", g);
    run(b, [&] { p_rowseg<<<g, 256>>>(y, 0); });
    snprintf(b, 64, "contig 1KB G=%d", g);
    run(b, [&] { p_rowseg<<<g, 256>>>(y, 1); });
    snprintf(b, 64, "rowseg shifted G=%d", g);
    run(b, [&] { p_rowseg<<<g, 256>>>(y, 2); });
    snprintf(b, 64, "lane-row 16B G=%d", g);
    run(b, [&] { p_lanerow<<<g, 256>>>(y); });
  }
  hipFree(y);
  return 0;
}
