// Calibration probe (not part of the product): f32 MFMA throughput on gfx950 for
// dependent single chains vs independent chains.  Built by tools/probe/Makefile.
#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CH>
__global__ __launch_bounds__(256) void p32(float* out, int iters) {
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c) for (int v = 0; v < 16; ++v) acc[c][v] = 0.f;
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  float s = 0.f;
  for (int c = 0; c < CH; ++c) for (int v = 0; v < 16; ++v) s += acc[c][v];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int CH>
__global__ __launch_bounds__(256) void p16(float* out, int iters) {
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) for (int v = 0; v < 4; ++v) acc[c][v] = 0.f;
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  float s = 0.f;
  for (int c = 0; c < CH; ++c) for (int v = 0; v < 4; ++v) s += acc[c][v];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

extern "C" int probe(int shape, int chains, int blocks, int iters, float* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define L(SH, C) if (shape == SH && chains == C) { p##SH<C><<<blocks, 256, 0, s>>>(out, iters); return 0; }
  L(32, 1) L(32, 2) L(32, 4) L(16, 1) L(16, 2) L(16, 4) L(16, 8)
  return -1;
}
