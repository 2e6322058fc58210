// Probe: cycles per step of a 4-accumulator FMA chain step as used by hmm_seg.hip's phase 1
// (m -> 16 FMAs (4 chains of 4) -> combine -> m), with the m operand broadcast by DPP row_newbcast
// (mode 0), plain VGPR operand (mode 1), DPP quad_perm (mode 2).  One wave per SIMD / two per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/dpp_lat.hip -o tools/probe/dpp_lat && ./tools/probe/dpp_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE, int N>
__device__ __forceinline__ float fm(float acc, float m, float p) {
  if constexpr (MODE == 0) asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(m), "v"(p), "i"(N));
  else if constexpr (MODE == 2) asm("v_fmac_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(m), "v"(p));
  else asm("v_fmac_f32 %0, %1, %2" : "+v"(acc) : "v"(m), "v"(p));
  return acc;
}

template <int MODE>
__global__ void probe(float* out, long long* cyc, int iters) {
  float m = threadIdx.x * 1e-3f, p0 = 0.5f, p1 = 0.25f, p2 = 0.125f, p3 = 0.0625f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    float a = 0.f, b = 0.f, c = 0.f, d = 0.f;
    asm volatile("s_nop 1");
    a = fm<MODE, 0>(a, m, p0); b = fm<MODE, 8>(b, m, p0); c = fm<MODE, 4>(c, m, p1); d = fm<MODE, 12>(d, m, p1);
    a = fm<MODE, 1>(a, m, p1); b = fm<MODE, 9>(b, m, p1); c = fm<MODE, 5>(c, m, p2); d = fm<MODE, 13>(d, m, p2);
    a = fm<MODE, 2>(a, m, p2); b = fm<MODE, 10>(b, m, p2); c = fm<MODE, 6>(c, m, p3); d = fm<MODE, 14>(d, m, p3);
    a = fm<MODE, 3>(a, m, p3); b = fm<MODE, 11>(b, m, p3); c = fm<MODE, 7>(c, m, p0); d = fm<MODE, 15>(d, m, p0);
    m = (threadIdx.x & 8) ? b + d : a + c;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = m;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 1 << 16);
  const int iters = 4096;
  for (int mode = 0; mode < 3; ++mode)
    for (int threads = 256; threads <= 512; threads *= 2) {
      for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0) probe<0><<<256, threads>>>(out, cyc, iters);
        if (mode == 1) probe<1><<<256, threads>>>(out, cyc, iters);
        if (mode == 2) probe<2><<<256, threads>>>(out, cyc, iters);
      }
      hipDeviceSynchronize();
      long long h[256];
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double s = 0;
      for (int i = 0; i < 256; ++i) s += h[i];
      printf("mode %d (%s) waves/SIMD %d: %.1f cycles per step\n", mode, mode == 0 ? "row_newbcast" : mode == 1 ? "plain" : "quad_perm",
             threads / 256, s / 256 / iters);
    }
  return 0;
}
