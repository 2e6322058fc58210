// Diagnostic probe (not product code): the clock the chip holds under a dense f32 MFMA loop
// shaped like the conv kernels' inner loop (ds_read_b128 operands from LDS holding random data,
// 4 independent 16x16x4 accumulators per wave), and the TFLOP/s it delivers.
//   clock = d(s_memtime) / d(s_memrealtime) * 100 MHz, stamped once per workgroup around the loop
//   (MI355X_MICROARCH.md, DVFS give-back item 6).
// build: hipcc --offload-arch=gfx950 -O3 -o mfma_clock mfma_clock.hip     run: ./mfma_clock [waves/SIMD]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) void mfma_loop(const float* __restrict__ src, int iters, float* out,
                                                   unsigned long long* stamps) {
  __shared__ float4 lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x)
    lds[i] = reinterpret_cast<const float4*>(src)[(blockIdx.x * 4096 + i) & ((1 << 18) - 1)];  // src: 2^18 float4
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f32x4 acc[4] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 b = lds[(lane + 64 * ((it + k) & 31)) & 4095];
      float4 a[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) a[nb] = lds[(lane + 64 * nb + 256 * k) & 4095];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nb].x, b.x, acc[nb], 0, 0, 0);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nb].y, b.y, acc[nb], 0, 0, 0);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nb].z, b.z, acc[nb], 0, 0, 0);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nb].w, b.w, acc[nb], 0, 0, 0);
    }
  }
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    stamps[blockIdx.x * 2] = t1 - t0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
  float s = 0.f;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) s += acc[nb][0] + acc[nb][1] + acc[nb][2] + acc[nb][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 2;  // waves per SIMD
  const int threads = 256 * wps, blocks = 256, iters = 4000;
  std::vector<float> h(1 << 20);
  srand(1);
  for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
  float *src, *out;
  unsigned long long* st;
  hipMalloc(&src, h.size() * 4);
  hipMalloc(&out, (size_t)blocks * threads * 4);
  hipMalloc(&st, blocks * 16);
  hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 200; ++w) mfma_loop<<<blocks, threads>>>(src, iters, out, st);  // > 2 s warm
  hipEventRecord(e0);
  const int reps = 20;
  for (int w = 0; w < reps; ++w) mfma_loop<<<blocks, threads>>>(src, iters, out, st);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return 1; }
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> hs(blocks * 2);
  hipMemcpy(hs.data(), st, blocks * 16, hipMemcpyDeviceToHost);
  std::vector<double> clk;
  for (int b = 0; b < blocks; ++b) clk.push_back(hs[2 * b] / (double)hs[2 * b + 1] * 0.1);  // GHz
  std::sort(clk.begin(), clk.end());
  const double flops = 2.0 * 16 * 16 * 4 * 64.0 * iters * (threads / 64) * (double)blocks * reps;  // 64 MFMAs/iter/wave
  printf("waves/SIMD %d: %.1f TFLOP/s f32 MFMA, in-kernel clock median %.3f GHz (min %.3f max %.3f), %.3f ms/launch\n",
         wps, flops / (ms * 1e-3) / 1e12, clk[blocks / 2], clk[0], clk[blocks - 1], ms / reps);
  return 0;
}
