// VQ nearest-neighbour quantization: idx[b,t] = argmin_k ||z[b,:,t] - c[k,:]||^2.
//
// Semantics (no reference code exists): pseudocode.txt:11
// `quantize(z_e, codebook)` and the hard-regime argmax of backtesting.py:154-155.
// Exact contract (oracle/hmm_ref.py, oracle/c/hmm_oracle.c): per k the distance is
// the fmaf chain over d = 0..Dv-1 of (z_d - c_kd)^2 from +0.0f, and the first k
// with the smallest distance wins.  The kernel evaluates exactly that chain.
//
// Design (cfg3: 4*N*Dv bytes in, 4*N out; 2 VALU ops per (n,k,d) -> VALU and
// HBM roofs are within 30% of each other, so both the load path and the
// VALU stream are kept dense):
//  * one wave = 128 consecutive positions, lane l owns positions n0+l and
//    n0+64+l; every z load is a coalesced 256-B wave access of the CF tensor;
//  * a block of KB codewords is staged in LDS once per workgroup and read
//    with wave-uniform float4 broadcasts: one ds_read_b128 feeds 16 VALU ops
//    (4 dims x 2 positions x {v_sub, v_fma});
//  * per lane 2*KB independent fma chains give ILP; z for a 16-dim chunk
//    stays in VGPRs and is reused across all KB codewords.
#include "kernels.h"

namespace vqhmm {

constexpr int VQ_DCH = 16;

template <int KB>
__global__ __launch_bounds__(256) void vq_argmin_kernel(const float* __restrict__ z, int64_t B, int Dv, int T,
                                                        const float* __restrict__ cb, int K, int ldc,
                                                        int32_t* __restrict__ idx, float* __restrict__ dmin) {
  extern __shared__ float4 cbs4[];
  float* cbs = reinterpret_cast<float*>(cbs4);  // [KB][ldc], ldc = Dv rounded up to 16
  const int64_t N = B * (int64_t)T;
  const int lane = threadIdx.x & 63;
  const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 128;
  const int64_t na = n0 + lane, nb = n0 + 64 + lane;
  const bool va = na < N, vb = nb < N;
  const int64_t ba = va ? na / T : 0, bb = vb ? nb / T : 0;
  const float* za = z + ba * (int64_t)Dv * T + (va ? na - ba * T : 0);
  const float* zb = z + bb * (int64_t)Dv * T + (vb ? nb - bb * T : 0);

  float best_a = __builtin_inff(), best_b = __builtin_inff();
  int arg_a = 0, arg_b = 0;
  for (int kb = 0; kb < K; kb += KB) {
    const int kn = min(KB, K - kb);
    __syncthreads();
    for (int i = threadIdx.x; i < KB * ldc; i += 256) {
      const int k = i / ldc, d = i - k * ldc;
      cbs[i] = (k < kn && d < Dv) ? cb[(int64_t)(kb + k) * Dv + d] : 0.0f;
    }
    __syncthreads();
    float acc_a[KB], acc_b[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) acc_a[k] = acc_b[k] = 0.0f;
    for (int dc = 0; dc < Dv; dc += VQ_DCH) {
      const int dn = min(VQ_DCH, Dv - dc);
      float zca[VQ_DCH], zcb[VQ_DCH];
      if (dn == VQ_DCH) {
#pragma unroll
        for (int d = 0; d < VQ_DCH; ++d) {
          zca[d] = va ? za[(int64_t)(dc + d) * T] : 0.0f;
          zcb[d] = vb ? zb[(int64_t)(dc + d) * T] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const float4* c4 = reinterpret_cast<const float4*>(cbs + k * ldc + dc);
#pragma unroll
          for (int q = 0; q < VQ_DCH / 4; ++q) {
            const float4 c = c4[q];
            const float cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float da = zca[4 * q + e] - cc[e];
              const float db = zcb[4 * q + e] - cc[e];
              acc_a[k] = __builtin_fmaf(da, da, acc_a[k]);
              acc_b[k] = __builtin_fmaf(db, db, acc_b[k]);
            }
          }
        }
      } else {  // ragged last chunk: still strictly d-ascending per chain
        for (int d = 0; d < dn; ++d) {
          const float zva = va ? za[(int64_t)(dc + d) * T] : 0.0f;
          const float zvb = vb ? zb[(int64_t)(dc + d) * T] : 0.0f;
#pragma unroll
          for (int k = 0; k < KB; ++k) {
            const float c = cbs[k * ldc + dc + d];
            const float da = zva - c, db = zvb - c;
            acc_a[k] = __builtin_fmaf(da, da, acc_a[k]);
            acc_b[k] = __builtin_fmaf(db, db, acc_b[k]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (k < kn) {
        if (acc_a[k] < best_a) { best_a = acc_a[k]; arg_a = kb + k; }
        if (acc_b[k] < best_b) { best_b = acc_b[k]; arg_b = kb + k; }
      }
    }
  }
  if (va) { idx[na] = arg_a; if (dmin) dmin[na] = best_a; }
  if (vb) { idx[nb] = arg_b; if (dmin) dmin[nb] = best_b; }
}

int launch_vq_argmin(const float* z, int64_t B, int64_t Dv, int64_t T, const float* cb, int64_t K,
                     int32_t* idx, float* dmin, hipStream_t s) {
  const int64_t N = B * T;
  if (N == 0) return VQHMM_OK;
  if (K <= 0 || Dv <= 0 || Dv > 2048 || T <= 0 || T > INT32_MAX) return VQHMM_EINVAL;
  const int ldc = (int)cdiv(Dv, VQ_DCH) * VQ_DCH;
  const dim3 grid((unsigned)cdiv(N, 512));
  int kb = K <= 4 ? 4 : K <= 8 ? 8 : K <= 16 ? 16 : 32;
  while (kb > 4 && (size_t)kb * ldc * 4 > 64 * 1024) kb >>= 1;
  const size_t lds = (size_t)kb * ldc * sizeof(float);
  if (lds > 64 * 1024) return VQHMM_EUNSUPPORTED;
  switch (kb) {
    case 4: vq_argmin_kernel<4><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
    case 8: vq_argmin_kernel<8><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
    case 16: vq_argmin_kernel<16><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
    default: vq_argmin_kernel<32><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
