// Prior.forward on the matrix cores (VQ_VAE_HMM_fixed.py:59-71): for every
// position (b, t), hid = relu(W1 u + b1) (TH), z = W2 hid + b2 (K*K), log_A[b, t, i, :] =
// log_softmax(z[i*K : i*K + K]).  This is the inference / API path (`model.prior(u)`); the training
// step computes the same MLP inside the ELBO head and never writes log_A.
//
// Every wave works alone on 16-position tiles (persistent, dealt CU-first):
//   hid^T (TH x 16)  = W1 (TH x U) @ u^T          on v_mfma_f32_16x16x4_f32, b1 as the accumulator start
//   z^T   (KK x 16)  = W2 (KK x TH) @ relu(hid^T)  KB = ceil(KK / 16) independent accumulator chains;
//                                                  the hid fragments ARE the B operand (no transpose)
//   row log_softmax from a wave-private LDS tile, one (position, row) per lane, stored as K contiguous
//   floats of log_A (coalesced across lanes).
// The weights are staged in LDS once per workgroup.  K*K <= 64, U <= 4, TH a multiple of 16 <= 256.
#include "kernels.h"
#include "prior_tile.h"

namespace vqhmm {

namespace {
template <int HB, int KB>
struct PriorLds {
  PriorW<HB, KB> w;
  float zS[4][16 * PriorW<HB, KB>::LDZ];
};
}  // namespace

template <int HB, int KB>
__global__ __launch_bounds__(256) void prior_mfma_kernel(PriorArgs p, int64_t ntiles) {
  using S = PriorLds<HB, KB>;
  constexpr int LDZ = PriorW<HB, KB>::LDZ;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int K = p.K, KK = K * K, U = p.U;
  prior_stage_weights<HB, KB>(sh.w, p.W1, p.b1, p.W2, K, U, tid, 256);
  f32x4 b2f[KB];
  prior_b2_frags<KB>(b2f, p.b2, KK, lg4);
  __syncthreads();
  float* zS = sh.zS[wave];
  const int64_t N = p.B * (int64_t)p.T;
  const int64_t stride = 4 * (int64_t)gridDim.x;
  for (int64_t tile = (int64_t)wave * gridDim.x + blockIdx.x; tile < ntiles; tile += stride) {
    // B operand of the hidden MFMA: u[position l16][channel lg4] (0 past U)
    const int64_t n = tile * 16 + l16;
    float ub = 0.f;
    if (n < N && lg4 < U) {
      const int64_t b = n / p.T;
      const int t = (int)(n - b * p.T);
      ub = p.u[b * (int64_t)U * p.T + lg4 * p.u_sc + (int64_t)t * p.u_st];
    }
    prior_tile<HB, KB>(sh.w, b2f, ub, l16, lg4, zS);
    __builtin_amdgcn_wave_barrier();
    for (int idx = lane; idx < 16 * K; idx += 64) {
      const int pos = idx / K, i = idx - pos * K;
      const int64_t np = tile * 16 + pos;
      if (np >= N) continue;
      prior_row_lsm(&zS[pos * LDZ + i * K], K, p.log_A + np * KK + i * K);
    }
    __builtin_amdgcn_wave_barrier();  // zS is rewritten by the next tile
  }
}

bool prior_mfma_supported(const PriorArgs& p) {
  return p.K >= 1 && p.K * p.K <= 64 && p.U >= 1 && p.U <= 4 && p.TH % 16 == 0 && p.TH >= 16 && p.TH <= 256;
}

template <int HB, int KB>
static int launch_pm(const PriorArgs& p, hipStream_t s) {
  const int64_t ntiles = cdiv(p.B * (int64_t)p.T, 16);
  const int64_t want = cdiv(ntiles, 4);
  const int64_t grid = want < 512 ? want : 512;
  prior_mfma_kernel<HB, KB><<<(unsigned)grid, 256, sizeof(PriorLds<HB, KB>), s>>>(p, ntiles);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

template <int HB>
static int launch_pm_k(const PriorArgs& p, hipStream_t s) {
  switch (prior_kb(p.K)) {
    case 1: return launch_pm<HB, 1>(p, s);
    case 2: return launch_pm<HB, 2>(p, s);
    default: return launch_pm<HB, 4>(p, s);
  }
}

int launch_prior_mfma(const PriorArgs& p, hipStream_t s) {
  if (!prior_mfma_supported(p)) return VQHMM_EUNSUPPORTED;
  if (p.B * (int64_t)p.T == 0) return VQHMM_OK;
  switch (p.TH / 16) {
    case 4: return launch_pm_k<4>(p, s);
    case 8: return launch_pm_k<8>(p, s);
    case 16: return launch_pm_k<16>(p, s);
    default: return VQHMM_EUNSUPPORTED;
  }
}

}  // namespace vqhmm
