// The Prior MLP on one 16-position tile (VQ_VAE_HMM_fixed.py:53-57,68-69), shared by
// prior.hip (log_A to HBM) and the fused Prior -> Viterbi kernel (prior_viterbi.hip, log_A to LDS) so
// that both produce the same bits for every (b, t, i, j):
//   hid^T (TH x 16) = W1 (TH x U) @ u^T           v_mfma_f32_16x16x4_f32, b1 as the accumulator start
//   z^T   (KK x 16) = W2 (KK x TH) @ relu(hid^T)   KB = ceil(KK / 16) independent accumulator chains;
//                                                 the hid fragments ARE the B operand (no transpose)
//   log_A row i = log_softmax(z[i*K : i*K + K])    one (position, row) per lane from a wave-private tile
// Contraction is pinned off in the row log_softmax (both files compile it the same way).
#pragma once
#include "common.h"

namespace vqhmm {

template <int HB, int KB>
struct PriorW {
  static constexpr int TH = HB * 16, KP2 = KB * 16;
  static constexpr int LDW2 = TH + 8;  // conflict-free b128 reads of W2 rows
  static constexpr int LDZ = KP2 + 4;  // z tile row stride
  float W2S[KP2 * LDW2];
  float W1S[TH * 8];  // [h][c]: W1 (c < U), b1 at c = 4
};

// block-cooperative weight staging (caller barriers afterwards)
template <int HB, int KB>
__device__ __forceinline__ void prior_stage_weights(PriorW<HB, KB>& w, const float* W1, const float* b1,
                                                    const float* W2, int K, int U, int tid, int nthr) {
  using S = PriorW<HB, KB>;
  constexpr int TH = S::TH;
  const int KK = K * K;
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < S::KP2 * S::LDW2; i += nthr) {
    const int ij = i / S::LDW2, h = i - ij * S::LDW2;
    w.W2S[i] = (ij < KK && h < TH) ? W2[(int64_t)ij * TH + h] : 0.f;
  }
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < TH * 8; i += nthr) {
    const int h = i >> 3, c = i & 7;
    w.W1S[i] = c < U ? W1[h * U + c] : (c == 4 ? b1[h] : 0.f);
  }
}

// this lane's b2 accumulator-start fragments (row ij = kb*16 + 4*lg4 + v)
template <int KB>
__device__ __forceinline__ void prior_b2_frags(f32x4* b2f, const float* b2, int KK, int lg4) {
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ij = kb * 16 + 4 * lg4 + v;
      b2f[kb][v] = ij < KK ? b2[ij] : 0.f;
    }
}

// z^T fragments of one tile; ub = u[position l16][channel lg4] (0 past U / past the data).
// Leaves the tile in zS[position][ij] (row stride LDZ) for prior_row_lsm.
template <int HB, int KB>
__device__ __forceinline__ void prior_tile(const PriorW<HB, KB>& w, const f32x4* b2f, float ub, int l16, int lg4,
                                           float* zS) {
  using S = PriorW<HB, KB>;
  f32x4 z[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) z[kb] = b2f[kb];
  // operands of hidden block hb: W1 column fragment, b1 accumulator start
  auto hid_ops = [&](int hb, float& w1, f32x4& c) {
    w1 = w.W1S[(hb * 16 + l16) * 8 + lg4];
#pragma unroll
    for (int v = 0; v < 4; ++v) c[v] = w.W1S[(hb * 16 + 4 * lg4 + v) * 8 + 4];
  };
  auto hid = [&](float w1, f32x4 c) {
    f32x4 h = mfma16x16x4(w1, ub, c);
#pragma unroll
    for (int v = 0; v < 4; ++v) h[v] = fmaxf(h[v], 0.f);
    return h;
  };
  auto w2_ops = [&](int hb, f32x4* w2v) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      w2v[kb] = *reinterpret_cast<const f32x4*>(&w.W2S[(kb * 16 + l16) * S::LDW2 + hb * 16 + 4 * lg4]);
  };
  // software-pipelined: block hb + 1's LDS operands are read while block hb's MFMAs run
  float w1;
  f32x4 c1, w2c[KB], w2n[KB];
  hid_ops(0, w1, c1);
  f32x4 hc = hid(w1, c1);
  w2_ops(0, w2c);
  if (HB > 1) hid_ops(1, w1, c1);
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
    if (hb + 1 < HB) w2_ops(hb + 1, w2n);
    const f32x4 hn = hb + 1 < HB ? hid(w1, c1) : hc;  // next block's hidden MFMA beside this one's
    if (hb + 2 < HB) hid_ops(hb + 2, w1, c1);
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) z[kb] = mfma16x16x4(w2c[kb][v], hc[v], z[kb]);
    hc = hn;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) w2c[kb] = w2n[kb];
  }
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) *reinterpret_cast<f32x4*>(&zS[l16 * S::LDZ + kb * 16 + 4 * lg4]) = z[kb];
}

// out[j] = zr[j] - logsumexp(zr[0..K)), j < K
__device__ __forceinline__ void prior_row_lsm(const float* zr, int K, float* out) {
#pragma clang fp contract(off)
  float m = -__builtin_inff();
  for (int j = 0; j < K; ++j) m = fmaxf(m, zr[j]);
  float s = 0.f;
  for (int j = 0; j < K; ++j) s += __expf(zr[j] - m);
  const float ls = m + __logf(s);
  for (int j = 0; j < K; ++j) out[j] = zr[j] - ls;
}

// KB for K*K transition logits (K*K <= 64)
__host__ __device__ constexpr int prior_kb(int K) { return (K * K + 15) / 16 <= 1 ? 1 : (K * K + 15) / 16 <= 2 ? 2 : 4; }

}  // namespace vqhmm
