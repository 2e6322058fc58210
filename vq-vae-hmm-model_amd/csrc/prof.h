// Phase-stamp profiling of persistent kernels (VQHMM_*_PROF builds; results unchanged): a kernel built
// with PROF > 0 writes s_memrealtime stamps (100 MHz) of workgroup w's phases into g_prof[w * 16 + k].
// One array per translation unit (internal linkage); vqhmm_debug_prof(which, ..) copies one of them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace vqhmm {
namespace {
__device__ unsigned long long g_prof[256 * 16];

template <int PROF>
__device__ __forceinline__ void stamp(int k) {
  if constexpr (PROF > 0) {
    if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memrealtime();
  }
}

__device__ __forceinline__ void stamp_if(bool on, int k) {
  if (on && threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memrealtime();
}

// the environment switch of one kernel family, read once; profiling build only (common.h VQHMM_PROF_ENV)
inline int prof_env_value(const char* e) { return e ? atoi(e) : 0; }
#ifdef VQHMM_PROFILING
#define prof_env(name) prof_env_value(getenv(name))
#else
#define prof_env(name) prof_env_value(nullptr)
#endif

inline int prof_copy(uint64_t* out, int64_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
}  // namespace
}  // namespace vqhmm
