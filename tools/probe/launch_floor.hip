// Probe: duration of a (near) empty kernel against its grid size and kernel-argument size, to price the
// fixed cost of the step's small launches (prologue, tail).  Timed by rocprofv3 --kernel-trace --stats.
// build: hipcc --offload-arch=gfx950 -O3 tools/probe/launch_floor.hip -o tools/probe/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { float* p; int pad[250]; };  // ~1 KB of kernel arguments

__global__ __launch_bounds__(256) void empty_small(float* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1.f;
}
__global__ __launch_bounds__(256) void empty_big(Big b) {
  if (b.p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) b.p[0] = (float)b.pad[threadIdx.x & 127];
}
__global__ __launch_bounds__(256) void one_load(const float* q, float* p) {  // one global load + store per thread
  const int i = blockIdx.x * 256 + threadIdx.x;
  p[i] = q[i] + 1.f;
}

int main() {
  float *p, *q;
  hipMalloc(&p, 4 << 20);
  hipMalloc(&q, 4 << 20);
  hipMemset(q, 0, 4 << 20);
  Big b{};
  b.p = nullptr;
  const unsigned grids[] = {64, 256, 512, 1024, 2048};
  for (int rep = 0; rep < 50; ++rep)
    for (unsigned g : grids) {
      empty_small<<<g, 256>>>(nullptr);
      empty_big<<<g, 256>>>(b);
      one_load<<<g, 256>>>(q, p);
    }
  hipDeviceSynchronize();
  // the same kernels replayed from a captured graph of five launches (the step's shape)
  hipStream_t st;
  hipStreamCreate(&st);
  hipGraph_t gr;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int k = 0; k < 5; ++k) empty_big<<<512, 256, 0, st>>>(b);
  hipStreamEndCapture(st, &gr);
  hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
  for (int rep = 0; rep < 50; ++rep) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  printf("done\n");
  return 0;
}
