// Device helpers shared by the strip kernels (strip.hip: forward / backward strips; strip_bwdw.hip: the
// backward strip with the six weight gradients folded in).  Header-only, like conv2_dev.h, so every
// translation unit compiles the very same epilogue arithmetic.
#pragma once
#include "conv2_dev.h"

namespace vqhmm {

namespace {
constexpr int ST_WIN = 128;                    // window rows: 8 MFMA row blocks, one per wave
constexpr int ST_HALO = 2;                     // inexact rows on each side
constexpr int ST_OWN = ST_WIN - 2 * ST_HALO;   // rows a strip stores
constexpr int ST_XR = ST_WIN + 4;              // rows of the shared x / q buffers (s0 - 2 .. s0 + 129)
constexpr int ST_XLD = 8;                      // their row stride
constexpr int ST_LDW = 72;                     // c2_ldx(64): 64-channel slots and weight images
constexpr int ST_LDF = 24;                     // the prologue's packed-front image row stride
constexpr int SB_LDE = 40;                     // c2_ldx(32): enc_conv2's dgrad input rows (dh2) and its image

// row_bt's validity test with 32-bit arithmetic (R < 2^31): PCL row r is a sequence position
__device__ __forceinline__ bool row_valid(int64_t r, int64_t R, int T) {
  if (r < 0 || r >= R) return false;
  const unsigned Tp = (unsigned)T + 2u, m = (unsigned)r % Tp;
  return m >= 1u && m <= (unsigned)T;
}

// A workgroup barrier for LDS data that leaves LDS DMA (global_load_lds, counted in vmcnt) in flight:
// lds_barrier()'s release fence makes the compiler drain vmcnt before the barrier whenever DMAs are
// outstanding.  Here each wave's LDS writes complete (lgkmcnt(0)) before s_barrier, and the "memory"
// clobber keeps the compiler's memory operations on their side of it; consumers of DMA'd data wait for
// their own DMAs (vmcnt) before the barrier that publishes them.
__device__ __forceinline__ void lds_barrier_dma() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void dma16(const float* src, float* dst) {
  __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(src), (__attribute__((address_space(3))) void*)dst,
                                   16, 0, 0);
}

// conv2_epilogue's ACT = 2 arithmetic (scale, no bias, ReLU-backward mask, pad rows 0) on a 64-wide
// block: rows r0 + l16, stored (PCL, 64 channels) for l16 in [slo, shi) when out is set, optionally to LDS
// rows xs (every row, or only row `only` when only >= 0), row 0 also to the row xlo and row 15 to the row
// xhi (when given)
__device__ __forceinline__ void mask_epi(f32x4 (&acc)[4], const float4 (&aux)[4], float sc, int64_t r0, int64_t R,
                                         int T, int lg4, int l16, int slo, int shi, float* out, float* xs, int xld,
                                         int only = -1, float* xlo = nullptr, float* xhi = nullptr) {
  const int64_t r = r0 + l16;
  const bool valid = row_valid(r, R, T);
  const bool st = out && l16 >= slo && l16 < shi && r < R;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const float av[4] = {aux[nb].x, aux[nb].y, aux[nb].z, aux[nb].w};
    f32x4 y;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float yy = acc[nb][v] * sc + 0.f;
      yy = av[v] > 0.f ? yy : 0.f;
      y[v] = valid ? yy : 0.f;
    }
    acc[nb] = y;
    if (st) *reinterpret_cast<f32x4*>(out + r * 64 + nb * 16 + 4 * lg4) = y;
    if (xs && (only < 0 || l16 == only)) *reinterpret_cast<f32x4*>(xs + l16 * xld + nb * 16 + 4 * lg4) = y;
    if (xlo && l16 == 0) *reinterpret_cast<f32x4*>(xlo + nb * 16 + 4 * lg4) = y;
    if (xhi && l16 == 15) *reinterpret_cast<f32x4*>(xhi + nb * 16 + 4 * lg4) = y;
  }
}

// the 64-channel mask rows r0 + l16 of a block (clamped into [0, R): rows outside are not stored)
__device__ __forceinline__ void load_mask(const float* m, int64_t r0, int64_t R, int lg4, int l16, float4 (&aux)[4]) {
  int64_t r = r0 + l16;
  r = r < 0 ? 0 : (r >= R ? R - 1 : r);
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) aux[nb] = *reinterpret_cast<const float4*>(m + r * 64 + nb * 16 + 4 * lg4);
}
}  // namespace

}  // namespace vqhmm
