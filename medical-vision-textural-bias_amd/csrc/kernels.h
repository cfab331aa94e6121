// kernels.h -- gfx950 kernels of the k-space filter passes and their launchers.
//
// Each pass kernel is compiled in its own translation unit (kern_*.hip), once per radix set
// (-DTB_RS=0 / 1), so the heavily unrolled FFT bodies build in parallel; texbias.hip (host
// side of the C ABI) calls the launchers declared at the bottom.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <unordered_map>

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
  int nbc;  // volume-channels of the launch (persistent compiled-plan kernels walk H * nbc units)
};

struct KspaceArgs {
  tb_plan_dev pl;
  cf* S;
  int bc0, C, T;
  int cofs;  // channel-volume index of blockIdx.y = 0 within ops (bc0 - first sample's bc)
  BatchOps ops;
  int nbc;   // channel-volumes of the launch (the persistent pass B walks nbc * tiles units)
};

struct SlabInvArgs {
  tb_plan_dev pl;
  const cf* S;
  float* y;
  int64_t sbc, sh, sw;
  int ypad, bc0, C;
  float scale;
  uint32_t* mm;
  int nbc;
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

// Compile-time slab plans (slab_ct.h, kern_slab_ct.hip): persistent passes A / C, grid from ncu.
bool slab_ct_supported(int W, int D);
hipError_t launch_slab_fwd_ct(const SlabFwdArgs& a, int ncu, hipStream_t st);
hipError_t launch_slab_inv_ct(const SlabInvArgs& a, int ncu, hipStream_t st);
// Compile-time pass-B plans (kspace_ct.h, kern_kspace_ct.hip): tile width kspace_ct_tile() columns.
bool kspace_ct_supported(int H);
int kspace_ct_tile(int ncols);
hipError_t launch_kspace_ct(const KspaceArgs& a, dim3 grid, int ncu, hipStream_t st);
bool kspace_ct_persistent(int ncols);  // launch_kspace_ct runs the persistent k_kspace_ct2p
// Half units and split spectra (slab_ct.h HalfPlan): passes A / C per (slab, row parity), two
// workgroups per CU; pass B finishes the W transform (kspace_ct.h b_mid_split).
bool slab_half_supported(int W, int D);
hipError_t launch_slab_fwd_half(const SlabFwdArgs& a, hipStream_t st);
hipError_t launch_slab_inv_half(const SlabInvArgs& a, hipStream_t st);
bool kspace_half_supported(int H, int W, int D);
hipError_t launch_kspace_half(const KspaceArgs& a, int ncu, hipStream_t st);

// Direct-DFT fallback (kern_generic.hip) for sizes the mixed-radix passes do not take: full complex
// spectrum in two ping-pong buffers S[2][nbc][H][W][D] (gen_workspace_bytes).
struct GenLaunch {
  tb_plan_dev pl;
  const float* x;
  const int64_t* xs;
  float* y;
  const int64_t* ys;
  cf* S;
  int ypad, bc0, C, nbc;  // bc0 = first sample * C; ops->s[i] = the run's i-th sample
  uint32_t* mm;
  const BatchOps* ops;
};
size_t gen_workspace_bytes(int H, int W, int D, int bc);
hipError_t launch_gen_filter(const GenLaunch& g, hipStream_t st);
hipError_t launch_gen_logabs(const GenLaunch& g, double* out, hipStream_t st);

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

// Wave-wide min / max on DPP lane moves (VALU, a few cycles each) instead of six dependent
// ds_bpermute round trips through the LDS pipe: quad swaps, half-row and row mirrors, then the
// gfx9 row broadcasts of lanes 15 and 31 (rows a broadcast does not write keep their own value);
// lane 63 ends with the result, read back as a wave-uniform value.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROW_MASK, 0xf, false));
}
template <class Op>
__device__ __forceinline__ float wave_reduce(float v, Op op) {
  v = op(v, dpp_f32<0xB1, 0xf>(v));   // quad_perm [1, 0, 3, 2]
  v = op(v, dpp_f32<0x4E, 0xf>(v));   // quad_perm [2, 3, 0, 1]
  v = op(v, dpp_f32<0x141, 0xf>(v));  // row_half_mirror
  v = op(v, dpp_f32<0x140, 0xf>(v));  // row_mirror
  v = op(v, dpp_f32<0x142, 0xa>(v));  // row_bcast:15 into rows 1, 3
  v = op(v, dpp_f32<0x143, 0xc>(v));  // row_bcast:31 into rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_min(float v) {
  return wave_reduce(v, [](float x, float y) { return fminf(x, y); });
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float x, float y) { return fmaxf(x, y); });
}

// Three-operand min / max (v_min3_f32 / v_max3_f32) without the canonicalising v_max_f32 x, x, x that
// fminf / fmaxf put on every operand the compiler cannot prove canonical (loop-carried running values,
// packed-math results): one instruction per two values folded in.  For the running min / max of
// arithmetic results (a quiet NaN operand is ignored, as by fminf).  max3_abs folds |b|, |c| in.
__device__ __forceinline__ float min3_raw(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max3_abs(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
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

// Last-arriver hand-off between the workgroups of one launch (they may sit on different XCDs, whose
// L2s are not coherent) without __threadfence(): its agent-scope release writes back the XCD's whole
// L2 (buffer_wbl2) from every workgroup -- 12 us at the end of pass C', 100+ us over the 2,048
// workgroups of the closed-form apply.  Instead the partial goes out as a device-scope atomic store,
// the workgroup waits for it (workgroup-scope release: s_waitcnt only) and counts itself in with a
// device-scope atomic; the last one reads the partials with device-scope atomic loads.
__device__ __forceinline__ void store_partial(float2* p, float2 v) {
  const uint64_t u = ((uint64_t)__float_as_uint(v.y) << 32) | (uint64_t)__float_as_uint(v.x);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 load_partial(const float2* p) {
  const uint64_t u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((uint32_t)u), __uint_as_float((uint32_t)(u >> 32)));
}
// Wait until every vector-memory operation this wave issued has completed.  A workgroup-scope
// release compiles to an lgkmcnt wait only, so without this an sc1 partial can still be in flight
// when the counter add lands.  Every wave that called store_partial runs it before the barrier
// that precedes arrive_last (the calling wave's own stores are drained inside arrive_last).
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// count the calling thread's workgroup in after its store_partial calls; true for the last of `total`
__device__ __forceinline__ bool arrive_last(uint32_t* cnt, uint32_t total) {
  drain_vmem();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  return __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
}

// Raise a kernel's dynamic-LDS limit to `bytes` (the launch's dynamic LDS) once per kernel: the
// kernels share one function type, so the cache is keyed by the kernel's address.  The request is
// the launch's own size -- 160 KiB plus a kernel's static LDS would be refused.
template <class K>
hipError_t allow_lds(K kern, size_t bytes) {
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> done;
  const void* f = reinterpret_cast<const void*>(kern);
  std::lock_guard<std::mutex> lk(mu);
  auto it = done.find(f);
  if (it != done.end() && it->second >= bytes) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) done[f] = bytes;
  return e;
}
template <class K>
hipError_t allow_full_lds(K kern) {
  return allow_lds(kern, 163840);
}
#endif

}  // namespace tb
