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

namespace vqhmm {

namespace {
template <int HB, int KB>
struct PriorLds {
  static constexpr int TH = HB * 16, KP2 = KB * 16;
  static constexpr int LDW2 = TH + 8;  // conflict-free b128 reads of W2 rows (as conv2's c2_ldx)
  static constexpr int LDZ = KP2 + 4;
  float W2S[KP2 * LDW2];
  float W1S[TH * 8];  // [h][c]: W1 (c < U), b1 at c = 4
  float zS[4][16 * LDZ];
};
}  // namespace

template <int HB, int KB>
__global__ __launch_bounds__(256) void prior_mfma_kernel(PriorArgs p, int64_t ntiles) {
  using S = PriorLds<HB, KB>;
  constexpr int TH = S::TH;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int K = p.K, KK = K * K, U = p.U;
  for (int i = tid; i < S::KP2 * S::LDW2; i += 256) {
    const int ij = i / S::LDW2, h = i - ij * S::LDW2;
    sh.W2S[i] = (ij < KK && h < TH) ? p.W2[(int64_t)ij * TH + h] : 0.f;
  }
  for (int i = tid; i < TH * 8; i += 256) {
    const int h = i >> 3, c = i & 7;
    sh.W1S[i] = c < U ? p.W1[h * U + c] : (c == 4 ? p.b1[h] : 0.f);
  }
  f32x4 b2f[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ij = kb * 16 + 4 * lg4 + v;
      b2f[kb][v] = ij < KK ? p.b2[ij] : 0.f;
    }
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
    f32x4 z[KB];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) z[kb] = b2f[kb];
    auto hid = [&](int hb) {
      const float w1 = sh.W1S[(hb * 16 + l16) * 8 + lg4];
      f32x4 c;
#pragma unroll
      for (int v = 0; v < 4; ++v) c[v] = sh.W1S[(hb * 16 + 4 * lg4 + v) * 8 + 4];
      f32x4 h = mfma16x16x4(w1, ub, c);
#pragma unroll
      for (int v = 0; v < 4; ++v) h[v] = fmaxf(h[v], 0.f);
      return h;
    };
    f32x4 hc = hid(0);
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
      f32x4 w2v[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        w2v[kb] = *reinterpret_cast<const f32x4*>(&sh.W2S[(kb * 16 + l16) * S::LDW2 + hb * 16 + 4 * lg4]);
      const f32x4 hn = hb + 1 < HB ? hid(hb + 1) : hc;  // next block's hidden MFMA beside this one's
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) z[kb] = mfma16x16x4(w2v[kb][v], hc[v], z[kb]);
      hc = hn;
    }
    // z^T fragments -> zS[position][ij], then one (position, row) per lane
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) *reinterpret_cast<f32x4*>(&zS[l16 * S::LDZ + kb * 16 + 4 * lg4]) = z[kb];
    __builtin_amdgcn_wave_barrier();
    for (int idx = lane; idx < 16 * K; idx += 64) {
      const int pos = idx / K, i = idx - pos * K;
      const int64_t np = tile * 16 + pos;
      if (np >= N) continue;
      const float* zr = &zS[pos * S::LDZ + i * K];
      float m = -__builtin_inff();
      for (int j = 0; j < K; ++j) m = fmaxf(m, zr[j]);
      float s = 0.f;
      for (int j = 0; j < K; ++j) s += __expf(zr[j] - m);
      const float ls = m + __logf(s);
      float* out = p.log_A + np * KK + i * K;
      for (int j = 0; j < K; ++j) out[j] = zr[j] - ls;
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
  const int kb = (p.K * p.K + 15) / 16;
  if (kb <= 1) return launch_pm<HB, 1>(p, s);
  if (kb <= 2) return launch_pm<HB, 2>(p, s);
  return launch_pm<HB, 4>(p, s);
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
