// Probe: HBM read rate of the forward-backward kernel's table-load pattern (hmm_seg.hip): every wave reads its
// own contiguous 16 KB (64 steps x 256 B), 512 workgroups x 8 waves (the cfg4 shard, 64 MB), all issued up
// front.  Modes: 0 = buffer_load_dword, one 256 B step per instruction (the kernel's form); 1 = the odd
// steps transposed within the step (as the kernel's lane map); 2 = buffer_load_dwordx4, four steps per
// instruction.  Each wave sums what it loaded (kept live) and writes one float.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/load_pattern.hip -o tools/probe/load_pattern && ./tools/probe/load_pattern
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang diagnostic ignored "-Wunused-result"

template <int MODE>
__global__ __launch_bounds__(512) void loads(const float* __restrict__ tab, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* base = tab + ((size_t)blockIdx.x * 8 + w) * 4096;  // 16 KB per wave
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 16384, 0x00020000);
  float acc = 0.f;
  if constexpr (MODE == 2) {
    float4 v[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int off = n * 1024 + lane * 16;
      v[n] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    }
#pragma unroll
    for (int n = 0; n < 16; ++n) acc += v[n].x + v[n].y + v[n].z + v[n].w;
  } else {
    const int ra = lane >> 3, cb = lane & 7;
    const int o0 = (ra * 8 + cb) * 4, o1 = MODE == 1 ? (cb * 8 + ra) * 4 : o0;
    float v[64];
#pragma unroll
    for (int u = 0; u < 64; ++u)
      v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (u & 1) ? o1 : o0, u * 256, 0));
#pragma unroll
    for (int u = 0; u < 64; ++u) acc += v[u];
  }
  out[(size_t)blockIdx.x * 512 + threadIdx.x] = acc;
}

int main() {
  const int nb = 512;
  const size_t n = (size_t)nb * 8 * 4096;
  float *tab, *out;
  hipMalloc(&tab, n * 4);
  hipMalloc(&out, (size_t)nb * 512 * 4);
  hipMemset(tab, 0, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"dword, one step per instruction", "dword, odd steps transposed", "dwordx4, 4 steps per instruction"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 3; ++mode) {
      float best = 1e9f;
      for (int it = 0; it < 20; ++it) {
        hipEventRecord(e0);
        if (mode == 0) loads<0><<<nb, 512>>>(tab, out);
        else if (mode == 1) loads<1><<<nb, 512>>>(tab, out);
        else loads<2><<<nb, 512>>>(tab, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
      }
      printf("mode %d (%s): %.2f us, %.2f TB/s\n", mode, names[mode], best * 1e3f, n * 4 / (best * 1e-3) / 1e12);
    }
  return 0;
}
