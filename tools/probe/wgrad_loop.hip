// Diagnostic probe (not product code): the weight-gradient body's inner loop in isolation — per wave 12
// accumulators of v_mfma_f32_16x16x4_f32 (4 output blocks x 3 taps) and, per 4-row step, 7 ds_read_b32
// operands (4 A + 3 B) read one step ahead into a second register set, as wgrad2.hip's compute lambda.
// Variant 0: that loop.  Variant 1: operands from registers only (no LDS reads: the MFMA issue floor).
// Variant 2: A operands as one ds_read_b128 per block per 4 steps ([n][row] image transposed to [row..]).
// Reports cycles per MFMA per SIMD (s_memtime, wave 0 of each workgroup) for W waves per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 -o wgrad_loop wgrad_loop.hip     run: ./wgrad_loop
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0)

template <int VAR>
__global__ __launch_bounds__(256) void loop(const float* __restrict__ src, int iters, float* out,
                                            unsigned long long* stamps) {
  __shared__ float lds[1][64 * 68 + 66 * 68];  // 35 KB: four workgroups fit a CU
  for (int i = threadIdx.x; i < 64 * 68 + 66 * 68; i += 256) lds[0][i] = src[(blockIdx.x * 977 + i) & ((1 << 18) - 1)];
  __syncthreads();
  const int lane = threadIdx.x & 63, lg4 = lane >> 4, l16 = lane & 15, wave = threadIdx.x >> 6;
  f32x4 acc[3][4] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (lane == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  const float* dys = lds[0];
  const float* xs = lds[0] + 64 * 68;
  float av[2][4], bv[2][3];
  auto load = [&](int st, float (&a)[4], float (&b)[3]) {
    const int rr = (st >> 2) * 16 + 4 * lg4 + (st & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = dys[rr * 68 + i * 16 + l16];
#pragma unroll
    for (int t = 0; t < 3; ++t) b[t] = xs[(rr + t) * 68 + wave * 16 + l16];
  };
  for (int it = 0; it < iters; ++it) {
    if constexpr (VAR == 1) {
#pragma unroll
      for (int st = 0; st < 16; ++st)
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[t][i] = MF((float)(st + i), (float)(t + it), acc[t][i]);
    } else if constexpr (VAR == 0) {
      load(0, av[0], bv[0]);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int cb = st & 1;
        if (st + 1 < 16) load(st + 1, av[cb ^ 1], bv[cb ^ 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[t][i] = MF(av[cb][i], bv[cb][t], acc[t][i]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      // A as float4 over 4 consecutive steps (rows 4 lg4 .. +3 of a 16-row slice): one ds_read_b128 per block
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        float4 a4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[i] = *reinterpret_cast<const float4*>(&dys[(i * 16 + l16) * 68 + sl * 16 + 4 * lg4]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float b[3];
          const int rr = sl * 16 + 4 * lg4 + e;
#pragma unroll
          for (int t = 0; t < 3; ++t) b[t] = xs[(rr + t) * 68 + wave * 16 + l16];
#pragma unroll
          for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float a = e == 0 ? a4[i].x : e == 1 ? a4[i].y : e == 2 ? a4[i].z : a4[i].w;
              acc[t][i] = MF(a, b[t], acc[t][i]);
            }
        }
      }
    }
  }
  if (lane == 0) {
    stamps[(blockIdx.x * 4 + wave) * 2] = __builtin_amdgcn_s_memtime() - t0;
    stamps[(blockIdx.x * 4 + wave) * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) s += acc[t][i][0] + acc[t][i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int VAR>
static void run(int wps, const float* src, float* out, unsigned long long* st) {
  const int blocks = 256 * wps, iters = 200;
  loop<VAR><<<blocks, 256>>>(src, iters, out, st);
  (void)hipDeviceSynchronize();
  loop<VAR><<<blocks, 256>>>(src, iters, out, st);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> raw(blocks * 8), h(blocks * 4), rt(blocks * 4);
  (void)hipMemcpy(raw.data(), st, raw.size() * 8, hipMemcpyDeviceToHost);
  for (int i = 0; i < blocks * 4; ++i) {
    h[i] = raw[2 * i];
    rt[i] = raw[2 * i + 1];
  }
  std::sort(h.begin(), h.end());
  std::sort(rt.begin(), rt.end());
  const double med = (double)h[h.size() / 2];
  printf("  clock %.2f GHz  ", med / (double)rt[rt.size() / 2] * 0.1);
  // per SIMD: wps waves each issuing iters * 192 MFMAs over med cycles
  printf("variant %d  waves/SIMD %d  cycles per MFMA per SIMD %.1f  (per wave %.1f)\n", VAR, wps,
         med / (iters * 192.0 * wps), med / (iters * 192.0));
}

int main() {
  float *src, *out;
  unsigned long long* st;
  (void)hipMalloc(&src, (1 << 18) * 4);
  (void)hipMalloc(&out, 256 * 4 * 256 * 4);
  (void)hipMalloc(&st, 256 * 4 * 4 * 8 * 2);
  std::vector<float> h(1 << 18);
  for (auto& v : h) v = (float)rand() / RAND_MAX;
  (void)hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (int w = 1; w <= 3; ++w) {
    run<0>(w, src, out, st);
    run<1>(w, src, out, st);
    run<2>(w, src, out, st);
  }
  return 0;
}
