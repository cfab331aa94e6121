// kernels.h -- gfx950 kernels of the k-space filter passes and their launchers.
//
// Each pass kernel is compiled in its own translation unit (kern_*.hip), once per radix set
// (-DTB_RS=0 / 1), so the heavily unrolled FFT bodies build in parallel; texbias.hip (host
// side of the C ABI) calls the launchers declared at the bottom.
#pragma once

#include <hip/hip_runtime.h>

#include "fft_core.h"
#include "sap_core.h"

namespace tb {

enum { RS_SMALL = 0, RS_ALL = 1 };

struct BatchOps {
  tb_sample_ops s[TB_MAX_BATCH];
};

struct SlabFwdArgs {
  tb_plan_dev pl;
  const float* x;
  int64_t sbc, sh, sw;
  cf* S;
  int bc0;
};

struct KspaceArgs {
  tb_plan_dev pl;
  cf* S;
  int bc0, C, T, pad;
  BatchOps ops;
};

struct SlabInvArgs {
  tb_plan_dev pl;
  const cf* S;
  float* y;
  int64_t sbc, sh, sw;
  int ypad, bc0, C;
  float scale;
  uint32_t* mm;
};

struct StatsArgs {
  tb_plan_dev pl;
  const cf* S;
  int bc0, C, T, pad;
  double* out;
  BatchOps ops;
};

constexpr int NT_SLAB = 512;
constexpr int NT_TILE = 256;

// Launchers (return hipError_t of the launch).  grid = (units, volume-channels).
template <int RS> hipError_t launch_slab_fwd(const SlabFwdArgs& a, dim3 grid, size_t lds, hipStream_t st);
template <int RS> hipError_t launch_kspace(const KspaceArgs& a, dim3 grid, size_t lds, hipStream_t st);
template <int RS> hipError_t launch_slab_inv(const SlabInvArgs& a, dim3 grid, size_t lds, hipStream_t st);
template <int RS> hipError_t launch_kspace_stats(const StatsArgs& a, dim3 grid, size_t lds, hipStream_t st);

#if defined(__HIPCC__)
struct DevCtx {
  int tid, nthreads;
  __device__ __forceinline__ void sync() { __syncthreads(); }
};

// Every kernel takes ONE argument struct and reads it through the kernarg segment pointer:
// dynamically indexed by-value parameters (the plan's radix lists, a sample's op program)
// are otherwise copied to per-lane scratch memory (2.4 KB per lane for the op programs).
template <class A>
__device__ __forceinline__ const A& kargs() {
  return *(const A*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block min/max -> atomic order-preserving keys (uses the first 2*NT/64 floats of smem after a barrier)
template <int NT>
__device__ __forceinline__ void block_minmax_atomic(float lo, float hi, float* red, uint32_t* mm) {
  lo = wave_min(lo);
  hi = wave_max(hi);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    red[wid] = lo;
    red[NT / 64 + wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NT / 64; ++w) {
      lo = fminf(lo, red[w]);
      hi = fmaxf(hi, red[NT / 64 + w]);
    }
    atomicMin(&mm[0], f2key(lo));
    atomicMax(&mm[1], f2key(hi));
  }
}

// Raise a kernel's dynamic-LDS limit to the CU's full 160 KiB once per process.
template <class K>
hipError_t allow_full_lds(K kern) {
  static const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  return e;
}
#endif

}  // namespace tb
