// Probe: operand / result lane layout of v_mfma_f32_4x4x1f32 (16 blocks of 4x4x1) and its issue cost and
// dependent latency, for a phase-1 transfer-matrix product of hmm_seg.hip on the matrix pipe.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma4x4.hip -o tools/probe/mfma4x4 && ./tools/probe/mfma4x4
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void layout(float* out, int mode) {
  const int l = threadIdx.x;
  const float a = mode == 0 ? (float)l : 1.f;
  const float b = mode == 0 ? 1.f : (float)l;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}

template <int DEP>
__global__ void timing(float* out, long long* cyc, int iters) {
  const int l = threadIdx.x;
  float a = 1e-3f * l, b = 0.5f;
  f4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (DEP == 1) {
        c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      } else {
        c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, b, c3, 0, 0, 0);
      }
    }
    a = c0[0] * 1e-9f + a;  // the next iteration's operand depends on the result: a full round trip
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* d;
  long long* dc;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&dc, 4096);
  float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    layout<<<1, 64>>>(d, mode);
    hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
    printf("mode %d (%s = lane index, other operand 1): lane: c[0] c[1] c[2] c[3]\n", mode, mode == 0 ? "A" : "B");
    for (int l = 0; l < 64; ++l) printf("  %2d: %4.0f %4.0f %4.0f %4.0f%s", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3], (l % 4 == 3) ? "\n" : "");
  }
  const int iters = 1000;
  long long hc[4];
  for (int rep = 0; rep < 2; ++rep) {
    timing<1><<<1, 64>>>(d, dc, iters);
    hipMemcpy(hc, dc, 8, hipMemcpyDeviceToHost);
    printf("dependent chain: %.2f cyc per mfma_f32_4x4x1f32 (8 per iteration, one accumulator)\n", (double)hc[0] / (iters * 8));
    timing<4><<<1, 64>>>(d, dc, iters);
    hipMemcpy(hc, dc, 8, hipMemcpyDeviceToHost);
    printf("4 accumulators:  %.2f cyc per mfma_f32_4x4x1f32 (32 per iteration)\n", (double)hc[0] / (iters * 32));
  }
  hipFree(d);
  hipFree(dc);
  return 0;
}
