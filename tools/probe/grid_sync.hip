// Probe: what a phase boundary costs on MI355X, as a kernel boundary against a grid-wide barrier inside one
// cooperative launch (the step is 5 dependent launches; at B = 128 each costs ~4.6 us even with no work,
// DESIGN §10).  Every phase writes X bytes (256 workgroups x 512 threads, float4 stores) so the boundary also
// has dirty L2 lines to publish to the next phase (other XCDs).
//   A: launches of writer, back to back                  -> per-launch time at X
//   B: cooperative kernel, P phases of (write X; grid.sync) -> per-phase time at X, from P = 9 vs P = 1
// Wall time from hipEvents over 200 repetitions.  hipLaunchCooperativeKernel refuses a grid that cannot be
// co-resident, so the barrier cannot wait for a workgroup that never starts.
// build: hipcc --offload-arch=gfx950 -O3 tools/probe/grid_sync.hip -o tools/probe/grid_sync
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <cstdio>

namespace cg = cooperative_groups;

__global__ __launch_bounds__(512) void writer(float4* p, int n4) {
  float4* q = p + (size_t)blockIdx.x * n4;
  for (int i = threadIdx.x; i < n4; i += 512) q[i] = make_float4((float)i, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(512) void coop(float4* p, int n4, int phases) {
  cg::grid_group g = cg::this_grid();
  float4* q = p + (size_t)blockIdx.x * n4;
  for (int ph = 0; ph < phases; ++ph) {
    for (int i = threadIdx.x; i < n4; i += 512) q[i] = make_float4((float)(i + ph), 0.f, 0.f, 0.f);
    g.sync();
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main() {
  const int G = 256, REPS = 200;
  float4* p;
  CK(hipMalloc(&p, (size_t)64 << 20));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t mbs[] = {0, 4, 16, 32};
  for (size_t mb : mbs) {
    int n4 = (int)((mb << 20) / 16 / G);
    // A: REPS launches of writer
    for (int w = 0; w < 20; ++w) writer<<<G, 512, 0, s>>>(p, n4);
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < REPS; ++r) writer<<<G, 512, 0, s>>>(p, n4);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ta;
    CK(hipEventElapsedTime(&ta, e0, e1));
    // B: cooperative, 1 and 9 phases
    float tb[2];
    const int ph[2] = {1, 9};
    for (int k = 0; k < 2; ++k) {
      int phases = ph[k];
      void* args[] = {&p, &n4, &phases};
      for (int w = 0; w < 5; ++w) CK(hipLaunchCooperativeKernel((void*)coop, dim3(G), dim3(512), args, 0, s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < REPS; ++r) CK(hipLaunchCooperativeKernel((void*)coop, dim3(G), dim3(512), args, 0, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&tb[k], e0, e1));
    }
    printf("X = %2zu MB per phase: launch %.2f us each | cooperative: 1 phase %.2f us, per extra phase %.2f us\n", mb,
           ta * 1e3f / REPS, tb[0] * 1e3f / REPS, (tb[1] - tb[0]) * 1e3f / REPS / 8);
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
