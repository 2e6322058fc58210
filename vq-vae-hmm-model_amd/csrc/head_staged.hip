// ELBO head for shapes the fused heads do not cover (large K: K^2 transition
// logits per position; wide U / TH / D).  Same math as head_mfma.hip
// (VQ_VAE_HMM_fixed.py:59-71 Prior, :106-137 loss), split into stages because
// log_A (B,T,K,K) no longer fits in registers:
//   1. hid  = relu(W1 u + b1)        1x1 conv over PCL rows (conv kernels)
//   2. lgA  = W2 hid + b2            1x1 conv, K^2 channels
//   3. L1   (this file) one wave per row, lane i = row i of log_A_t:
//           log_softmax, transition term w_t sum q_{t-1,i} q_{t,j} log_A_t[i][j],
//           nx_t[i] = sum_j log_A_t[i][j] q_{t,j}   (the t -> t+1 term of dq_{t-1}),
//           dqc_t[j] = sum_i q_{t-1,i} log_A_t[i][j] (the t-1 -> t term of dq_t),
//           d lgA (log_softmax backward) written in place over lgA
//   4. L2   (this file) one thread per row: recon NLL, entropy, init, dq, loss
//           partials (fixed-order block sums, deterministic)
//   5. dhid = (W2^T dlgA) * relu'(hid); dW2, db2, dW1, db1 by the wgrad kernels.
#include <algorithm>

#include "kernels.h"

namespace vqhmm {

template <int KM>
__global__ __launch_bounds__(256) void head_l1_kernel(StagedHeadArgs a) {
  __shared__ float qcS[4][KM];
  __shared__ float qpS[4][KM];
  __shared__ float laS[4][KM][KM + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = a.K, KK = K * K, LDA = ld4(KK), LQ = ld4(K);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.R; r += nw) {
    int64_t b;
    int t;
    const bool valid = row_bt(r, a.R, a.T, b, t);
    float* row = a.lgA + r * LDA;
    if (!valid) {  // pad rows: zero gradient rows (the wgrad / dgrad sums run over all rows)
      for (int e = lane; e < LDA; e += 64) row[e] = 0.f;
      if (lane < LQ) { a.nx[r * LQ + lane] = 0.f; a.dqc[r * LQ + lane] = 0.f; }
      if (lane == 0) a.trw[r] = 0.f;
      continue;
    }
    const int64_t L = a.lengths[b];
    const float w = (t >= 1 && t < L) ? 1.f : 0.f;
    if (lane < KM) {
      qcS[wave][lane] = lane < K ? a.q[r * LQ + lane] : 0.f;
      qpS[wave][lane] = lane < K ? a.q[(r - 1) * LQ + lane] : 0.f;  // row r-1 is a zero pad row at t = 0
    }
    __builtin_amdgcn_wave_barrier();
    float la[KM];
    float tri = 0.f, nxi = 0.f, qp = 0.f, sq = 0.f;
    if (lane < K) {
      const float* src = row + lane * K;
      float m = -__builtin_inff();
#pragma unroll
      for (int j = 0; j < KM; ++j) {
        la[j] = j < K ? src[j] : -__builtin_inff();
        m = fmaxf(m, la[j]);
      }
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < KM; ++j) s += j < K ? __expf(la[j] - m) : 0.f;
      const float ls = m + __logf(s);
      qp = qpS[wave][lane];
#pragma unroll
      for (int j = 0; j < KM; ++j) {
        if (j < K) {
          la[j] -= ls;
          const float qc = qcS[wave][j];
          nxi = fmaf(la[j], qc, nxi);
          sq += qc;
          laS[wave][lane][j] = la[j];
        }
      }
      tri = qp * nxi;
    }
    __builtin_amdgcn_wave_barrier();
    const float tr = wave_sum(tri);
    if (lane < K) a.nx[r * LQ + lane] = nxi;
    else if (lane < LQ) a.nx[r * LQ + lane] = 0.f;
    if (lane == 0) a.trw[r] = w * tr;
    // dqc_j = sum_i q_{t-1,i} log_A[i][j]  (lane j, column of the LDS copy)
    if (lane < LQ) {
      float d = 0.f;
      if (lane < K)
        for (int i = 0; i < K; ++i) d = fmaf(qpS[wave][i], laS[wave][i][lane], d);
      a.dqc[r * LQ + lane] = w * d;
    }
    // log_softmax backward of d tr / d log_A = cpri w q_{t-1,i} q_{t,j}
    if (lane < K) {
      const float ci = -a.beta / loss_norm_batch(a.norm, a.B) * w * qp;
      const float rs = ci * sq;
      float* dst = row + lane * K;
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (j < K) dst[j] = ci * qcS[wave][j] - __expf(la[j]) * rs;
    }
    if (lane < LDA - KK) row[KK + lane] = 0.f;
    __builtin_amdgcn_wave_barrier();
  }
}

// Sum over the 32 lanes of one parity (lane & 1) on the VALU: DPP xor 2 / row_ror:4 / row_ror:8 keep the
// parity, then the permlane swaps; no LDS round trip (ds_bpermute was 5 per value, 16 values per row).
__device__ __forceinline__ float parity_sum_dpp(float v) {
  v += __builtin_bit_cast(float, dpp_u32<0x4E>(__builtin_bit_cast(uint32_t, v)));   // quad_perm [2,3,0,1]
  v += __builtin_bit_cast(float, dpp_u32<0x124>(__builtin_bit_cast(uint32_t, v)));  // row_ror:4
  v += __builtin_bit_cast(float, dpp_u32<0x128>(__builtin_bit_cast(uint32_t, v)));  // row_ror:8
  float2 r = pair16(v);
  v = r.x + r.y;
  r = pair32(v);
  return r.x + r.y;
}
__device__ __forceinline__ float xor1_dpp(float v) {
  return __builtin_bit_cast(float, dpp_u32<0xB1>(__builtin_bit_cast(uint32_t, v)));  // quad_perm [1,0,3,2]
}

// head_l1 for 8 < K <= 32, one wave per row with every load and store a whole contiguous row: lane (i, h) =
// (l >> 1, l & 1) holds log_A_t[i][16 h .. 16 h + 15] (the old lane-per-i form walked each i row with a
// K-float stride per lane: 2.6 ms at cfg3).  Row reductions pair lanes (xor 1); the column sums dqc_j =
// sum_i q_{t-1,i} log_A[i][j] run over the 32 lanes of a half (parity_sum_dpp).  V4: K % 4 == 0
// (float4 rows).
template <bool V4>
__global__ __launch_bounds__(256) void head_l1_wide_kernel(StagedHeadArgs a) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // row math on SALU
  const int K = a.K, KK = K * K, LDA = ld4(KK), LQ = ld4(K);
  const int i = lane >> 1, h = lane & 1, j0 = 16 * h;
  const bool irow = i < K;
  const float cpri = -a.beta / loss_norm_batch(a.norm, a.B);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.R; r += nw) {
    int64_t b;
    int t;
    const bool valid = row_bt_fast(r, a.R, a.T, b, t);
    float* row = a.lgA + r * LDA;
    if (!valid) {  // pad rows: zero gradient rows (the wgrad / dgrad sums run over all rows)
      for (int e = lane; e < LDA; e += 64) row[e] = 0.f;
      if (lane < LQ) { a.nx[r * LQ + lane] = 0.f; a.dqc[r * LQ + lane] = 0.f; }
      if (lane == 0) a.trw[r] = 0.f;
      continue;
    }
    const int64_t L = a.lengths[b];
    const float w = (t >= 1 && t < L) ? 1.f : 0.f;
    float la[16], qc[16];
    if constexpr (V4) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bool in = irow && j0 + 4 * g < K;
        const float4 v = in ? *reinterpret_cast<const float4*>(row + i * K + j0 + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 c = j0 + 4 * g < K ? *reinterpret_cast<const float4*>(a.q + r * LQ + j0 + 4 * g)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        la[4 * g] = v.x; la[4 * g + 1] = v.y; la[4 * g + 2] = v.z; la[4 * g + 3] = v.w;
        qc[4 * g] = c.x; qc[4 * g + 1] = c.y; qc[4 * g + 2] = c.z; qc[4 * g + 3] = c.w;
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = j0 + jj;
        la[jj] = (irow && j < K) ? row[i * K + j] : 0.f;
        qc[jj] = j < K ? a.q[r * LQ + j] : 0.f;
      }
    }
    // log_softmax of row i (lanes 2i, 2i + 1)
    float m = -__builtin_inff();
#pragma unroll
    for (int jj = 0; jj < 16; ++jj)
      if (j0 + jj < K) m = fmaxf(m, la[jj]);
    m = fmaxf(m, xor1_dpp(m));
    float se = 0.f;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj)
      if (j0 + jj < K) se += __expf(la[jj] - m);
    se += xor1_dpp(se);
    const float ls = m + __logf(se);
    const float qp = irow ? a.q[(r - 1) * LQ + i] : 0.f;  // row r - 1 is a zero pad row at t = 0
    float nxi = 0.f, sq = 0.f;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      la[jj] -= ls;
      if (j0 + jj < K) {
        nxi = fmaf(la[jj], qc[jj], nxi);
        sq += qc[jj];
      }
    }
    nxi += xor1_dpp(nxi);
    sq += xor1_dpp(sq);
    // transition term sum_i q_{t-1,i} nx_i (each i counted once: h = 0 lanes)
    const float tri = parity_sum_dpp((irow && h == 0) ? qp * nxi : 0.f);
    if (h == 0 && i < LQ) a.nx[r * LQ + i] = irow ? nxi : 0.f;
    if (lane == 0) a.trw[r] = w * tri;  // lane 0 (h = 0) holds the sum over every i
    // dqc_j = w sum_i q_{t-1,i} log_A[i][j]: over the 32 lanes of this half
    float d[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) d[jj] = irow ? qp * la[jj] : 0.f;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) d[jj] = parity_sum_dpp(d[jj]);
    if (i == 0) {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj)
        if (j0 + jj < LQ) a.dqc[r * LQ + j0 + jj] = j0 + jj < K ? w * d[jj] : 0.f;
    }
    // log_softmax backward of d tr / d log_A = cpri w q_{t-1,i} q_{t,j}, in place over the row
    const float ci = cpri * w * qp, rs = ci * sq;
    float g[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) g[jj] = ci * qc[jj] - __expf(la[jj]) * rs;
    if constexpr (V4) {
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        if (irow && j0 + 4 * q4 < K)
          *reinterpret_cast<float4*>(row + i * K + j0 + 4 * q4) = make_float4(g[4 * q4], g[4 * q4 + 1], g[4 * q4 + 2], g[4 * q4 + 3]);
    } else {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj)
        if (irow && j0 + jj < K) row[i * K + j0 + jj] = g[jj];
    }
    for (int e = KK + lane; e < LDA; e += 64) row[e] = 0.f;
  }
}

// head_l1 for K = 16 / 32 with every wave-instruction on log_A a contiguous 1 KiB: lane l holds float4 number
// 64 g + l of the row-major K x K block (g < K^2 / 256), i.e. row i = (64 g + l) / (K / 4), columns
// 4 (l % (K / 4)) .. + 3.  A row's K / 4 lanes are adjacent (DPP quad / half-mirror sums); the column sums
// dqc_j run over the lanes with the same l % (K / 4) (row_ror + permlane swaps).  head_l1_wide's lane (i, h)
// form touched 64 separate 64-B segments per wave-instruction (0.94 ms at cfg3 for 3.57 GB, 3.8 TB/s).
template <int LPR>
__device__ __forceinline__ float row_sum_dpp(float v) {  // over the LPR (4 or 8) adjacent lanes of a row
  v += xor1_dpp(v);
  v += __builtin_bit_cast(float, dpp_u32<0x4E>(__builtin_bit_cast(uint32_t, v)));     // quad_perm [2,3,0,1]
  if constexpr (LPR == 8)
    v += __builtin_bit_cast(float, dpp_u32<0x141>(__builtin_bit_cast(uint32_t, v)));  // row_half_mirror
  return v;
}
template <int LPR>
__device__ __forceinline__ float row_max_dpp(float v) {
  v = fmaxf(v, xor1_dpp(v));
  v = fmaxf(v, __builtin_bit_cast(float, dpp_u32<0x4E>(__builtin_bit_cast(uint32_t, v))));
  if constexpr (LPR == 8) v = fmaxf(v, __builtin_bit_cast(float, dpp_u32<0x141>(__builtin_bit_cast(uint32_t, v))));
  return v;
}
template <int LPR>
__device__ __forceinline__ float col_sum_dpp(float v) {  // over the 64 / LPR lanes with the same lane % LPR
  if constexpr (LPR == 4)
    v += __builtin_bit_cast(float, dpp_u32<0x124>(__builtin_bit_cast(uint32_t, v)));  // row_ror:4
  v += __builtin_bit_cast(float, dpp_u32<0x128>(__builtin_bit_cast(uint32_t, v)));    // row_ror:8
  float2 r = pair16(v);
  v = r.x + r.y;
  r = pair32(v);
  return r.x + r.y;
}

template <int KP>
__global__ __launch_bounds__(256) void head_l1_pow2_kernel(StagedHeadArgs a) {
  constexpr int LPR = KP / 4, G = KP * KP / 256, KK = KP * KP;  // LDA = KK, LQ = KP
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // row math on SALU
  const int c0 = 4 * (lane % LPR);
  const bool lead = lane % LPR == 0;
  const float cpri = -a.beta / loss_norm_batch(a.norm, a.B);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.R; r += nw) {
    int64_t b;
    int t;
    const bool valid = row_bt_fast(r, a.R, a.T, b, t);
    float* row = a.lgA + r * KK;
    if (!valid) {  // pad rows: zero gradient rows (the wgrad / dgrad sums run over all rows)
#pragma unroll
      for (int g = 0; g < G; ++g) *reinterpret_cast<float4*>(row + 256 * g + 4 * lane) = make_float4(0.f, 0.f, 0.f, 0.f);
      if (lane < LPR) {
        *reinterpret_cast<float4*>(a.nx + r * KP + 4 * lane) = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(a.dqc + r * KP + 4 * lane) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (lane == 0) a.trw[r] = 0.f;
      continue;
    }
    float4 v[G];
    float qp[G];
#pragma unroll
    for (int g = 0; g < G; ++g) v[g] = *reinterpret_cast<const float4*>(row + 256 * g + 4 * lane);
    const float4 c = *reinterpret_cast<const float4*>(a.q + r * KP + c0);
#pragma unroll
    for (int g = 0; g < G; ++g) qp[g] = a.q[(r - 1) * KP + (64 * g + lane) / LPR];  // row r - 1: zero pad at t = 0
    const int64_t L = a.lengths[b];
    const float w = (t >= 1 && t < L) ? 1.f : 0.f;
    const float qc[4] = {c.x, c.y, c.z, c.w};
    const float sq = row_sum_dpp<LPR>((qc[0] + qc[1]) + (qc[2] + qc[3]));  // sum_j q_{t,j}
    float tri = 0.f, d[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float la[4] = {v[g].x, v[g].y, v[g].z, v[g].w};
      const float m = row_max_dpp<LPR>(fmaxf(fmaxf(la[0], la[1]), fmaxf(la[2], la[3])));
      float se = 0.f;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) se += __expf(la[cc] - m);
      const float ls = m + __logf(row_sum_dpp<LPR>(se));
      float nxi = 0.f;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        la[cc] -= ls;
        nxi = fmaf(la[cc], qc[cc], nxi);
        d[cc] = fmaf(qp[g], la[cc], d[cc]);
      }
      nxi = row_sum_dpp<LPR>(nxi);
      const int i = (64 * g + lane) / LPR;
      if (lead) {
        a.nx[r * KP + i] = nxi;
        tri = fmaf(qp[g], nxi, tri);  // transition term sum_i q_{t-1,i} nx_i, each i once
      }
      // log_softmax backward of d tr / d log_A = cpri w q_{t-1,i} q_{t,j}, in place over the row
      const float ci = cpri * w * qp[g], rs = ci * sq;
      *reinterpret_cast<float4*>(row + 256 * g + 4 * lane) =
          make_float4(ci * qc[0] - __expf(la[0]) * rs, ci * qc[1] - __expf(la[1]) * rs,
                      ci * qc[2] - __expf(la[2]) * rs, ci * qc[3] - __expf(la[3]) * rs);
    }
    tri = wave_sum_dpp(tri);
    if (lane == 0) a.trw[r] = w * tri;
    // dqc_j = w sum_i q_{t-1,i} log_A[i][j]
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) d[cc] = col_sum_dpp<LPR>(d[cc]);
    if (lane < LPR)
      *reinterpret_cast<float4*>(a.dqc + r * KP + c0) = make_float4(w * d[0], w * d[1], w * d[2], w * d[3]);
  }
}

__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, dpp_u32<0xB1>(__builtin_bit_cast(uint32_t, v))));
  v = fmaxf(v, __builtin_bit_cast(float, dpp_u32<0x4E>(__builtin_bit_cast(uint32_t, v))));
  v = fmaxf(v, __builtin_bit_cast(float, dpp_u32<0x141>(__builtin_bit_cast(uint32_t, v))));
  v = fmaxf(v, __builtin_bit_cast(float, dpp_u32<0x128>(__builtin_bit_cast(uint32_t, v))));
  float2 r = pair16(v);
  v = fmaxf(r.x, r.y);
  r = pair32(v);
  return fmaxf(r.x, r.y);
}

// head_l2: one wave per row, lane = channel (D <= 64 recon channels, K <= 64 states): every load and store is a whole
// contiguous row (the thread-per-row form read each row's channels 16 B apart per lane: 3.2 ms at cfg3); the
// row's log-sum-exp and <q, log q> are wave reductions (DPP + permlane, a fixed order).
// 16 waves per workgroup, RPW rows per wave per iteration (rows r0, r0 + nw, ...): the grid is capped at
// head_grid(R) workgroups (one loss partial each), so the memory-level parallelism has to come from inside
// the workgroup; cfg3 head_l2 (A/B on one box, rocprofv3 averages): one row per 4-wave workgroup
// 0.62 ms; 4 rows x 4 waves 0.39-0.42 (173 VGPRs); with the row math on the scalar unit (81 VGPRs)
// 256 x 4 / 1024 x 2 / 1024 x 4 / 512 x 4 / 1024 x 8 = 0.416 / 0.279 / 0.258 / 0.264 / 0.300 ms
constexpr int L2_NT = 1024, RPW = 4;

__global__ __launch_bounds__(L2_NT) void head_l2_kernel(StagedHeadArgs a) {
  __shared__ double red[4][L2_NT];
  __shared__ unsigned long long cnt;
  // wave index in an SGPR: the row index math and the per-row lengths / trw loads then run on the scalar unit
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int K = a.K, D = a.D, LQ = ld4(K), LP = ld4(2 * D), LX = ld4(D);
  if (tid == 0) cnt = a.norm ? (unsigned long long)a.norm[0] : 0ull;
  __syncthreads();
  {  // valid positions (the recon normaliser mask.sum() * C, VQ_VAE_HMM_fixed.py:120)
    unsigned long long c = 0;
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int64_t b = tid; !a.norm && b < a.B; b += L2_NT) {
      const int64_t L = a.lengths[b];
      c += (unsigned long long)(L <= 0 ? 0 : (L < a.T ? L : a.T));
    }
    atomicAdd(&cnt, c);
  }
  __syncthreads();
  const float inv_n = 1.0f / fmaxf((float)(cnt * (unsigned long long)D), 1.0f);
  const float cpri = -a.beta / loss_norm_batch(a.norm, a.B), cent = a.beta / loss_norm_batch(a.norm, a.B);
  const float lpk = lane < K ? a.log_pi[lane] : 0.f;
  float s_rec = 0.f, s_init = 0.f, s_tr = 0.f, s_ent = 0.f;
  // every load of a row group issued before any of its arithmetic and none gated on the lengths load: one row
  // per wave left ~200 dependent load -> reduce -> store rounds per wave at cfg3 (0.62 ms, latency-bound);
  // masked rows load but do not compute, as before
  const int64_t nw = (int64_t)gridDim.x * (L2_NT / 64);
  for (int64_t r0 = (int64_t)blockIdx.x * (L2_NT / 64) + wave; r0 < a.R; r0 += nw * RPW) {
    int64_t rr[RPW], L[RPW];
    int tt[RPW];
    bool ok[RPW], valid[RPW];
    float lg[RPW], qk[RPW], dqc[RPW], nxv[RPW], trw[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int64_t r = r0 + i * nw;
      int64_t b = 0;
      int t = 0;
      rr[i] = r;
      ok[i] = r < a.R;
      valid[i] = row_bt_fast(r, a.R, a.T, b, t);
      tt[i] = t;
      L[i] = valid[i] ? a.lengths[b] : 0;
      const bool vk = valid[i] && lane < K;
      lg[i] = ok[i] && lane < K ? a.logits[r * LQ + lane] : -__builtin_inff();
      qk[i] = ok[i] && lane < K ? a.q[r * LQ + lane] : 0.f;
      dqc[i] = vk ? a.dqc[r * LQ + lane] : 0.f;
      nxv[i] = vk ? a.nx[(r + 1) * LQ + lane] : 0.f;
      trw[i] = valid[i] ? a.trw[r] : 0.f;
    }
    // recon NLL, lane c = channel (c, c + 64, ...)
    for (int c = lane; c < D; c += 64) {
      float mu[RPW], lv[RPW], xv[RPW];
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int64_t r = rr[i];
        mu[i] = valid[i] ? a.par[r * LP + c] : 0.f;
        lv[i] = valid[i] ? a.par[r * LP + D + c] : 0.f;
        xv[i] = valid[i] ? a.x[r * LX + c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        float dmu = 0.f, dlv = 0.f;
        if (valid[i] && tt[i] < L[i]) {
          const float ev = __expf(lv[i]);
          const float var = (ev < 1e-8f ? 1e-8f : ev)  /* clamp(min=1e-8), NaN stays NaN */;
          const float df = mu[i] - xv[i];
          const float r2 = df * df / var;
          s_rec += 0.5f * (__logf(6.2831855f * var) + r2);
          dmu = df / var * inv_n;
          dlv = (ev >= 1e-8f) ? 0.5f * (1.f - r2) * inv_n : 0.f;
        }
        if (a.need_grad && ok[i]) {
          a.dpar[rr[i] * LP + c] = dmu;
          a.dpar[rr[i] * LP + D + c] = dlv;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      if (!ok[i]) continue;
      const int64_t r = rr[i];
      const int t = tt[i];
      const bool m = valid[i] && t < L[i];
      if (a.need_grad)
        for (int c = 2 * D + lane; c < LP; c += 64) a.dpar[r * LP + c] = 0.f;  // pad channels
      // entropy of q = softmax(logits) and its logits gradient, lane k = state
      const float mx = wave_max_dpp(lg[i]);
      const float lse = mx + __logf(wave_sum_dpp(lane < K ? __expf(lg[i] - mx) : 0.f));
      const float f = wave_sum_dpp(lane < K ? qk[i] * (lg[i] - lse) : 0.f);
      if (m && lane == 0) s_ent -= f;
      if (valid[i] && lane == 0) s_tr += trw[i];
      const float wn = (valid[i] && t + 1 < L[i]) ? 1.f : 0.f;  // weight of the t -> t+1 transition
      if (lane < LQ) {
        float dl = 0.f, dq = 0.f;
        if (valid[i] && lane < K) {
          if (m) dl = cent * qk[i] * ((lg[i] - lse) - f);
          dq = cpri * (dqc[i] + wn * nxv[i]);  // dqc already carries w_t
          if (t == 0) {
            dq = fmaf(cpri, lpk, dq);
            s_init = fmaf(qk[i], lpk, s_init);
          }
        }
        if (a.need_grad) {
          a.dlx[r * LQ + lane] = dl;
          a.dqx[r * LQ + lane] = dq;
        }
      }
    }
  }
  red[0][tid] = s_rec;
  red[1][tid] = s_init;
  red[2][tid] = s_tr;
  red[3][tid] = s_ent;
  __syncthreads();
  for (int st = L2_NT / 2; st > 0; st >>= 1) {
    if (tid < st)
      for (int i = 0; i < 4; ++i) red[i][tid] += red[i][tid + st];
    __syncthreads();
  }
  if (tid < 4) a.part[blockIdx.x * 4 + tid] = red[tid][0];
}

// q summed over the t = 0 rows (init term gradient of log_prior), one chunk: thread (part, k) sums sequences
// b = part, part + P, ... (P = 256 / ld4(K) parts, loads independent), the parts combined in a fixed order
// (was one thread per k over all B: 2048 dependent loads, 0.64 ms at cfg3)
__global__ __launch_bounds__(256) void head_q0_kernel(const float* q, int64_t B, int T, int K, float* q0) {
  __shared__ float part[256];
  const int L = ld4(K), P = 256 / L, k = threadIdx.x % L, ph = threadIdx.x / L;
  float s = 0.f;
  if (ph < P) {
#pragma unroll 8
    for (int64_t b = ph; b < B; b += P) s += q[(b * (T + 2) + 1) * L + k];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  if ((int)threadIdx.x < K) {
    float v = 0.f;
    for (int h = 0; h < P; ++h) v += part[h * L + threadIdx.x];
    q0[threadIdx.x] = v;
  }
}

__global__ void log_softmax_small_kernel(const float* v, int K, float* out) {
  if (threadIdx.x != 0) return;
  float m = -__builtin_inff();
  for (int k = 0; k < K; ++k) m = fmaxf(m, v[k]);
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += __expf(v[k] - m);
  const float l = m + __logf(s);
  for (int k = 0; k < K; ++k) out[k] = v[k] - l;
}

bool staged_head_supported(int K) { return K >= 1 && K <= 64; }  // lane = state (head_l1 / head_l2)

int launch_staged_head(const StagedHeadArgs& a, int l2grid, hipStream_t s) {
  if (!staged_head_supported(a.K)) return VQHMM_EUNSUPPORTED;
  log_softmax_small_kernel<<<1, 64, 0, s>>>(a.log_prior, a.K, a.log_pi);
  VQHMM_LAUNCH_CHECK();
  const unsigned g1 = (unsigned)std::min<int64_t>(cdiv(a.R, 4), 2048);
  if (a.K <= 8) head_l1_kernel<16><<<g1, 256, 0, s>>>(a);
  else if (a.K == 32) head_l1_pow2_kernel<32><<<g1, 256, 0, s>>>(a);
  else if (a.K == 16) head_l1_pow2_kernel<16><<<g1, 256, 0, s>>>(a);
  else if (a.K <= 32 && a.K % 4 == 0) head_l1_wide_kernel<true><<<g1, 256, 0, s>>>(a);
  else if (a.K <= 32) head_l1_wide_kernel<false><<<g1, 256, 0, s>>>(a);
  else head_l1_kernel<64><<<g1, 256, 0, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  head_l2_kernel<<<l2grid, L2_NT, 0, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  if (a.need_grad) {
    head_q0_kernel<<<1, 256, 0, s>>>(a.q, a.B, a.T, a.K, a.q0);
    VQHMM_LAUNCH_CHECK();
  }
  return VQHMM_OK;
}

}  // namespace vqhmm
