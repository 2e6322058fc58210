// Diagnostic probe (not product code): shader-clock cycles per step of the forward-backward
// linear-tier chain (hmm.hip) on one wave per SIMD, for the two reduction axes of K = 8 and for
// 1, 2 and 4 independent chains interleaved in one wave.
//   build: hipcc --offload-arch=gfx950 -O3 -o chain_lat chain_lat.hip     run: ./chain_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ float dppf(float v, int) { return v; }
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float2 pair16(float x) {
  float a = x, b = x;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return make_float2(a, b);
}
__device__ __forceinline__ float2 pair32(float x) {
  float a = x, b = x;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return make_float2(a, b);
}
__device__ __forceinline__ float red_inner(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  return v;
}
__device__ __forceinline__ float red_outer(float v) {
  v += dpp<0x128>(v);
  const float2 a = pair16(v);
  v = a.x + a.y;
  const float2 b = pair32(v);
  return b.x + b.y;
}

template <bool INNER>
__device__ __forceinline__ float red_max(float v) {
  if (INNER) {
    v = fmaxf(v, dpp<0xB1>(v));
    v = fmaxf(v, dpp<0x4E>(v));
    return fmaxf(v, dpp<0x141>(v));
  }
  v = fmaxf(v, dpp<0x128>(v));
  const float2 a = pair16(v);
  v = fmaxf(a.x, a.y);
  const float2 b = pair32(v);
  return fmaxf(b.x, b.y);
}

// the linear tier's step as in hmm.hip: + rescale every 4th step, range tracking, LDS store
template <int LEVEL>
__global__ __launch_bounds__(64) void full_chain(const float* __restrict__ m, int steps, float* out,
                                                 unsigned long long* stamps) {
  __shared__ float vb[16 * 8];
  const int lane = threadIdx.x;
  float x = 1.f + lane * 1e-3f, lo = 1.f, hi = 1.f;
  float mv[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) mv[s] = m[(s & 7) * 64 + lane];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < steps; it += 16) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool inner = s & 1;
      const float v = x * mv[s];
      int k = 0;
      if (LEVEL >= 1 && s % 4 == 0) k = __builtin_amdgcn_frexp_expf(inner ? red_max<true>(x) : red_max<false>(x));
      float y = inner ? red_inner(v) : red_outer(v);
      if (LEVEL >= 1 && s % 4 == 0) y = __builtin_amdgcn_ldexpf(y, -k);
      if (LEVEL >= 2) {
        lo = fminf(lo, y);
        hi = fmaxf(hi, y);
      }
      x = y;
      if (LEVEL >= 3) vb[s * 8 + (inner ? lane / 8 : lane % 8)] = x;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = x + lo + hi + vb[lane];
  if (lane == 0) stamps[blockIdx.x] = t1 - t0;
}

// MODE 0: inner steps only, 1: outer only, 2: alternating; NC independent chains
template <int MODE, int NC>
__global__ __launch_bounds__(64) void chain(const float* __restrict__ m, int steps, float* out,
                                            unsigned long long* stamps) {
  const int lane = threadIdx.x;
  float x[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) x[c] = 1.f + lane * 1e-3f + c;
  float mv[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) mv[s] = m[s * 64 + lane];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < steps; it += 8) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float v = x[c] * mv[s];
        const bool inner = MODE == 0 || (MODE == 2 && (s & 1));
        x[c] = inner ? red_inner(v) : red_outer(v);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) acc += x[c];
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) stamps[blockIdx.x] = t1 - t0;
}

template <int MODE, int NC>
static void run(const char* name, const float* m, float* out, unsigned long long* st, int steps) {
  chain<MODE, NC><<<256, 64>>>(m, steps, out, st);
  chain<MODE, NC><<<256, 64>>>(m, steps, out, st);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 256; ++i) s += h[i];
  printf("%-28s %6.1f cycles/step (per chain-step %6.1f)\n", name, s / 256 / steps, s / 256 / steps / NC);
}

template <int LEVEL>
static void runf(const char* name, const float* m, float* out, unsigned long long* st, int steps) {
  full_chain<LEVEL><<<256, 64>>>(m, steps, out, st);
  full_chain<LEVEL><<<256, 64>>>(m, steps, out, st);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 256; ++i) s += h[i];
  printf("%-28s %6.1f cycles/step\n", name, s / 256 / steps);
}

int main() {
  float *m, *out;
  unsigned long long* st;
  hipMalloc(&m, 8 * 64 * 4);
  hipMalloc(&out, 256 * 64 * 4);
  hipMalloc(&st, 256 * 8);
  float hm[512];
  for (int i = 0; i < 512; ++i) hm[i] = 0.125f * (1.f + (i % 7) * 1e-3f);
  hipMemcpy(m, hm, sizeof(hm), hipMemcpyHostToDevice);
  const int steps = 1 << 16;
  run<0, 1>("inner, 1 chain", m, out, st, steps);
  run<1, 1>("outer, 1 chain", m, out, st, steps);
  run<2, 1>("alternating, 1 chain", m, out, st, steps);
  run<2, 2>("alternating, 2 chains", m, out, st, steps);
  run<2, 4>("alternating, 4 chains", m, out, st, steps);
  runf<0>("full: chain only", m, out, st, steps);
  runf<1>("full: + rescale", m, out, st, steps);
  runf<2>("full: + range", m, out, st, steps);
  runf<3>("full: + LDS store", m, out, st, steps);
  return 0;
}
