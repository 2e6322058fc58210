// Fused ELBO head: everything of VAE_HMM.compute_loss (VQ_VAE_HMM_fixed.py:106-137)
// that is not a convolution, forward AND backward, in one pass over the rows:
//   * Prior.forward (:59-71): MLP U -> TH (ReLU) -> K*K, row log_softmax -> log_A,
//     recomputed per row in registers (log_A is never written to HBM),
//   * recon Gaussian NLL (:118-120) and d/d(mu, logvar),
//   * mean-field HMM prior term init + transitions (:123-131) and d/dq,
//     d/dlog_A -> through log_softmax -> MLP weight gradients,
//   * entropy (:134-135) and its d/dlogits.
// Per-block partial sums / weight-gradient partials go to slabs that a
// fixed-order reduction sums (deterministic).
//
// Tile = 255 rows of the PCL layout per 256-thread block (thread 255 builds the
// halo row r0+255, whose log_A the transition t -> t+1 of the last row needs).
#include <algorithm>

#include "kernels.h"

namespace vqhmm {


constexpr int HP = 255;  // useful rows per tile

// log_A[t] for one row, in registers: la[i*K + j].
template <int KM, int UM>
__device__ __forceinline__ void prior_row(const HeadArgs& a, const float* uv, float* la) {
  const int KK = a.K * a.K;
#pragma unroll
  for (int ij = 0; ij < KM * KM; ++ij) la[ij] = (ij < KK) ? a.b2[ij] : 0.f;
  for (int h = 0; h < a.TH; ++h) {
    float hv = a.b1[h];
#pragma unroll
    for (int c = 0; c < UM; ++c)
      if (c < a.U) hv = fmaf(a.W1[h * a.U + c], uv[c], hv);
    hv = relu_f(hv);
#pragma unroll
    for (int ij = 0; ij < KM * KM; ++ij)
      if (ij < KK) la[ij] = fmaf(a.W2[(int64_t)ij * a.TH + h], hv, la[ij]);
  }
#pragma unroll
  for (int i = 0; i < KM; ++i) {
    if (i >= a.K) break;
    float m = -__builtin_inff();
#pragma unroll
    for (int j = 0; j < KM; ++j)
      if (j < a.K) m = fmaxf(m, la[i * a.K + j]);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < KM; ++j)
      if (j < a.K) s += __expf(la[i * a.K + j] - m);
    const float ls = m + __logf(s);
#pragma unroll
    for (int j = 0; j < KM; ++j)
      if (j < a.K) la[i * a.K + j] -= ls;
  }
}

template <int KM, int UM>
__global__ __launch_bounds__(256) void elbo_head_kernel(HeadArgs a) {
  __shared__ float qS[(HP + 2) * KM];       // rows r0-1 .. r0+HP
  __shared__ float laS[(HP + 1) * KM * KM]; // rows r0 .. r0+HP (log_A, then dlog-logits)
  __shared__ float uS[(HP + 1) * UM];
  __shared__ int wS[HP + 2];                // transition weight w_t of rows r0 .. r0+HP
  __shared__ double red[4][256];
  __shared__ float lpS[KM];
  __shared__ unsigned long long cntS;

  const int tid = threadIdx.x;
  const int K = a.K, KK = K * K, D = a.D;
  const float Bn = loss_norm_batch(a.norm, a.B);
  const float cpri = -a.beta / Bn;  // d loss / d (init + trans)[b]
  const float cent = a.beta / Bn;   // d loss / d (sum q*log q)

  // log_pi = log_softmax(log_prior); valid-count for the recon normaliser
  if (tid == 0) {
    float m = -__builtin_inff();
    for (int k = 0; k < K; ++k) m = fmaxf(m, a.log_prior[k]);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += __expf(a.log_prior[k] - m);
    const float l = m + __logf(s);
    for (int k = 0; k < K; ++k) lpS[k] = a.log_prior[k] - l;
    cntS = a.norm ? (unsigned long long)a.norm[0] : 0ull;
  }
  __syncthreads();
  {
    unsigned long long c = 0;
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int64_t b = tid; !a.norm && b < a.B; b += 256) {
      const int64_t L = a.lengths[b];
      c += (unsigned long long)(L <= 0 ? 0 : (L < a.T ? L : a.T));
    }
    atomicAdd(&cntS, c);
  }
  __syncthreads();
  const float ncount = fmaxf((float)(cntS * (unsigned long long)D), 1.0f);
  const float inv_n = 1.0f / ncount;

  float s_rec = 0.f, s_ent = 0.f, s_tr = 0.f, s_init = 0.f;
  float q0acc[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) q0acc[k] = 0.f;
  // phase-3 ownership: thread -> hidden unit h, row phase g
  const int HPAD = a.TH <= 64 ? 64 : (a.TH <= 128 ? 128 : 256);
  const int G = 256 / HPAD;
  const int h = tid % HPAD, g = tid / HPAD;
  float gW2[KM * KM], gW1[UM], gb1 = 0.f, gb2 = 0.f;
#pragma unroll
  for (int i = 0; i < KM * KM; ++i) gW2[i] = 0.f;
#pragma unroll
  for (int i = 0; i < UM; ++i) gW1[i] = 0.f;
  float w2c[KM * KM], w1r[UM], b1h = 0.f;
  if (h < a.TH) {
#pragma unroll
    for (int i = 0; i < KM * KM; ++i) w2c[i] = i < KK ? a.W2[(int64_t)i * a.TH + h] : 0.f;
#pragma unroll
    for (int c = 0; c < UM; ++c) w1r[c] = c < a.U ? a.W1[h * a.U + c] : 0.f;
    b1h = a.b1[h];
  }

  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * HP;
    __syncthreads();
    // ---------------- phase 1: thread = row r0 + tid (tid 255 = halo row)
    {
      const int64_t r = r0 + tid;
      int64_t b;
      int t;
      const bool valid = row_bt(r, a.R, a.T, b, t);
      const int64_t L = valid ? a.lengths[b] : 0;
      const bool m = valid && t < L;
      wS[tid + 1] = (valid && t >= 1 && t < L) ? 1 : 0;
      float uv[UM];
#pragma unroll
      for (int c = 0; c < UM; ++c) uv[c] = (valid && c < a.U) ? a.u[r * ld4(a.U) + c] : 0.f;
#pragma unroll
      for (int c = 0; c < UM; ++c) uS[tid * UM + c] = uv[c];
      float la[KM * KM];
      prior_row<KM, UM>(a, uv, la);
#pragma unroll
      for (int ij = 0; ij < KM * KM; ++ij) laS[tid * KM * KM + ij] = la[ij];
#pragma unroll
      for (int k = 0; k < KM; ++k) qS[(tid + 1) * KM + k] = (valid && k < K) ? a.q[r * ld4(K) + k] : 0.f;
      if (tid == 0) {
        const int64_t rp = r0 - 1;
        int64_t bp;
        int tpv;
        const bool vp = row_bt(rp, a.R, a.T, bp, tpv);
#pragma unroll
        for (int k = 0; k < KM; ++k) qS[k] = (vp && k < K) ? a.q[rp * ld4(K) + k] : 0.f;
      }
      if (tid < HP && r < a.R) {
        // recon NLL (:118-120)
        for (int c = 0; c < D; ++c) {
          float dmu = 0.f, dlv = 0.f;
          if (m) {
            const float mu = a.par[r * ld4(2 * D) + c];
            const float lv = a.par[r * ld4(2 * D) + D + c];
            const float xv = a.x[r * ld4(D) + c];
            const float ev = __expf(lv);
            const float var = (ev < 1e-8f ? 1e-8f : ev)  /* clamp(min=1e-8), NaN stays NaN */;
            const float df = mu - xv;
            const float r2 = df * df / var;
            s_rec += 0.5f * (__logf(6.2831855f * var) + r2);
            dmu = df / var * inv_n;
            dlv = (ev >= 1e-8f) ? 0.5f * (1.f - r2) * inv_n : 0.f;
          }
          if (a.need_grad) {
            a.dpar[r * ld4(2 * D) + c] = dmu;
            a.dpar[r * ld4(2 * D) + D + c] = dlv;
          }
        }
        if (a.need_grad)
          for (int c = 2 * D; c < ld4(2 * D); ++c) a.dpar[r * ld4(2 * D) + c] = 0.f;
        // entropy (:134-135): sum_k q log_softmax
        float lg[KM], qv[KM];
        float mx = -__builtin_inff();
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          lg[k] = (valid && k < K) ? a.logits[r * ld4(K) + k] : 0.f;
          qv[k] = qS[(tid + 1) * KM + k];
          if (k < K) mx = fmaxf(mx, lg[k]);
        }
        float se = 0.f;
#pragma unroll
        for (int k = 0; k < KM; ++k)
          if (k < K) se += __expf(lg[k] - mx);
        const float lse = mx + __logf(se);
        float f = 0.f;
#pragma unroll
        for (int k = 0; k < KM; ++k)
          if (k < K) f = fmaf(qv[k], lg[k] - lse, f);
        if (m) s_ent -= f;
        if (a.need_grad) {
#pragma unroll
          for (int k = 0; k < KM; ++k)
            if (k < ld4(K)) a.dlx[r * ld4(K) + k] = (m && k < K) ? cent * qv[k] * ((lg[k] - lse) - f) : 0.f;
        }
        // init term (:123), unmasked, t == 0
        if (valid && t == 0) {
#pragma unroll
          for (int k = 0; k < KM; ++k)
            if (k < K) {
              s_init = fmaf(qv[k], lpS[k], s_init);
              q0acc[k] += qv[k];
            }
        }
      }
    }
    if (tid == 0) {
      int64_t bp;
      int tpv;
      const int64_t rp = r0 - 1;
      const bool vp = row_bt(rp, a.R, a.T, bp, tpv);
      wS[0] = (vp && tpv >= 1 && tpv < a.lengths[bp]) ? 1 : 0;
    }
    __syncthreads();
    // ---------------- phase 2a: transitions; dq for this row
    float dlA[KM * KM];
    if (tid < HP && r0 + tid < a.R) {
      const int64_t r = r0 + tid;
      const float* qp = qS + tid * KM;        // q[t-1]
      const float* qc = qS + (tid + 1) * KM;  // q[t]
      const float* qn = qS + (tid + 2) * KM;  // q[t+1]
      const float* la = laS + tid * KM * KM;
      const float* lan = laS + (tid + 1) * KM * KM;
      const float w = (float)wS[tid + 1];
      const float wn = (float)wS[tid + 2];
      float tr = 0.f;
      float dq[KM];
#pragma unroll
      for (int j = 0; j < KM; ++j) dq[j] = 0.f;
#pragma unroll
      for (int i = 0; i < KM; ++i) {
        if (i >= K) break;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
          if (j >= K) break;
          const float l = la[i * K + j];
          tr = fmaf(qp[i] * qc[j], l, tr);
          dq[j] = fmaf(qp[i], l, dq[j]);                         // from transition t-1 -> t
          dlA[i * K + j] = cpri * w * qp[i] * qc[j];
        }
      }
      s_tr += w * tr;
      if (a.need_grad) {
        int64_t b;
        int t;
        const bool valid = row_bt(r, a.R, a.T, b, t);
#pragma unroll
        for (int j = 0; j < KM; ++j) {
          if (j >= K) break;
          float nx = 0.f;  // from transition t -> t+1: sum_j' q[t+1, j'] log_A[t+1, j, j']
#pragma unroll
          for (int jj = 0; jj < KM; ++jj)
            if (jj < K) nx = fmaf(qn[jj], lan[j * K + jj], nx);
          float v = cpri * (w * dq[j] + wn * nx);
          if (valid && t == 0) v = fmaf(cpri, lpS[j], v);
          a.dqx[r * ld4(K) + j] = valid ? v : 0.f;
        }
        for (int j = K; j < ld4(K); ++j) a.dqx[r * ld4(K) + j] = 0.f;
      }
    }
    if (!a.need_grad) continue;
    __syncthreads();
    // ---------------- phase 2b: d log_A -> d transition logits (log_softmax backward), in place
    if (tid < HP) {
      float* la = laS + tid * KM * KM;
#pragma unroll
      for (int i = 0; i < KM; ++i) {
        if (i >= K) break;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < KM; ++j)
          if (j < K) s += dlA[i * K + j];
#pragma unroll
        for (int j = 0; j < KM; ++j)
          if (j < K) la[i * K + j] = dlA[i * K + j] - __expf(la[i * K + j]) * s;
      }
    }
    __syncthreads();
    // ---------------- phase 3: MLP weight gradients, thread = hidden unit h
    if (h < a.TH) {
      for (int row = g; row < HP; row += G) {
        if (r0 + row >= a.R) break;
        const float* uv = uS + row * UM;
        const float* dl = laS + row * KM * KM;
        float pre = b1h;
#pragma unroll
        for (int c = 0; c < UM; ++c) pre = fmaf(w1r[c], uv[c], pre);
        const float hv = relu_f(pre);
        float dh = 0.f;
#pragma unroll
        for (int ij = 0; ij < KM * KM; ++ij) {
          if (ij < KK) {
            const float d = dl[ij];
            dh = fmaf(w2c[ij], d, dh);
            gW2[ij] = fmaf(d, hv, gW2[ij]);
          }
        }
        dh = pre > 0.f ? dh : 0.f;
        gb1 += dh;
#pragma unroll
        for (int c = 0; c < UM; ++c) gW1[c] = fmaf(dh, uv[c], gW1[c]);
      }
    }
    if (tid < KK) {
      for (int row = 0; row < HP; ++row) {
        if (r0 + row >= a.R) break;
        gb2 += laS[row * KM * KM + tid];
      }
    }
  }

  // ---------------- block reductions -> slabs
  __syncthreads();
  red[0][tid] = s_rec;
  red[1][tid] = s_init;
  red[2][tid] = s_tr;
  red[3][tid] = s_ent;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st)
      for (int i = 0; i < 4; ++i) red[i][tid] += red[i][tid + st];
    __syncthreads();
  }
  if (tid < 4) a.part[blockIdx.x * 4 + tid] = red[tid][0];
  if (!a.need_grad) return;
  // q0 sums: K values
  for (int k = 0; k < K; ++k) {
    __syncthreads();
    float qv0 = 0.f;
#pragma unroll
    for (int kk = 0; kk < KM; ++kk)
      if (kk == k) qv0 = q0acc[kk];
    red[0][tid] = qv0;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (tid < st) red[0][tid] += red[0][tid + st];
      __syncthreads();
    }
    if (tid == 0) a.slab_q0[blockIdx.x * K + k] = (float)red[0][0];
  }
  // MLP grads: combine the G row phases in fixed order (phase 0 += phase 1, 2, ...)
  float* pS = laS;  // reuse: [HPAD][LDP] (fits: HPAD*LDP <= (HP+1)*KM*KM)
  const int LDP = KM * KM + UM + 1;
  for (int gg = 1; gg < G; ++gg) {
    __syncthreads();
    if (g == gg) {
#pragma unroll
      for (int i = 0; i < KM * KM; ++i) pS[h * LDP + i] = gW2[i];
#pragma unroll
      for (int c = 0; c < UM; ++c) pS[h * LDP + KM * KM + c] = gW1[c];
      pS[h * LDP + KM * KM + UM] = gb1;
    }
    __syncthreads();
    if (g == 0) {
      const float* o = pS + h * LDP;
#pragma unroll
      for (int i = 0; i < KM * KM; ++i) gW2[i] += o[i];
#pragma unroll
      for (int c = 0; c < UM; ++c) gW1[c] += o[KM * KM + c];
      gb1 += o[KM * KM + UM];
    }
  }
  if (g == 0 && h < a.TH) {
    float* sW2 = a.slab_W2 + (int64_t)blockIdx.x * KK * a.TH;
#pragma unroll
    for (int ij = 0; ij < KM * KM; ++ij)
      if (ij < KK) sW2[(int64_t)ij * a.TH + h] = gW2[ij];
    float* sW1 = a.slab_W1 + (int64_t)blockIdx.x * a.TH * a.U;
#pragma unroll
    for (int c = 0; c < UM; ++c)
      if (c < a.U) sW1[h * a.U + c] = gW1[c];
    a.slab_b1[(int64_t)blockIdx.x * a.TH + h] = gb1;
  }
  if (tid < KK) a.slab_b2[(int64_t)blockIdx.x * KK + tid] = gb2;
}

int head_grid(int64_t R) {
  const int64_t ntiles = cdiv(R, HP);
  return (int)(ntiles < 512 ? ntiles : 512);
}

bool fused_head_supported(const HeadArgs& a) {
  return head_mfma_supported(a) || (a.K <= 8 && a.U <= 8 && a.TH <= 256 && a.D <= 16);
}

int launch_head(const HeadArgs& a0, int grid, hipStream_t s) {
  HeadArgs a = a0;
  a.ntiles = cdiv(a.R, HP);
  if (a.R == 0) return VQHMM_OK;
  if (head_mfma_supported(a)) return launch_head_mfma(a, grid, s);
  if (a.K > 8 || a.U > 8 || a.TH > 256 || a.D > 16) return VQHMM_EUNSUPPORTED;
  if (a.K <= 4)
    elbo_head_kernel<4, 8><<<grid, 256, 0, s>>>(a);
  else
    elbo_head_kernel<8, 8><<<grid, 256, 0, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ---------------------------------------------------------------- Prior.forward

template <int KM, int UM>
__global__ __launch_bounds__(256) void prior_fwd_kernel(PriorArgs p) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= p.B * p.T) return;
  const int64_t b = n / p.T;
  const int t = (int)(n - b * p.T);
  HeadArgs a{};
  a.K = p.K; a.U = p.U; a.TH = p.TH;
  a.W1 = p.W1; a.b1 = p.b1; a.W2 = p.W2; a.b2 = p.b2;
  float uv[UM];
#pragma unroll
  for (int c = 0; c < UM; ++c) uv[c] = c < p.U ? p.u[b * (int64_t)p.U * p.T + c * p.u_sc + t * p.u_st] : 0.f;
  float la[KM * KM];
  prior_row<KM, UM>(a, uv, la);
  const int KK = p.K * p.K;
#pragma unroll
  for (int ij = 0; ij < KM * KM; ++ij)
    if (ij < KK) p.log_A[n * KK + ij] = la[ij];
}

// Any K <= 64, TH <= 1024: one wave per position; hidden layer and the K*K
// logits staged in LDS, then lane i log_softmaxes row i of log_A.
__global__ __launch_bounds__(256) void prior_fwd_wave_kernel(PriorArgs p) {
  __shared__ float hS[4][1024];
  __shared__ float zS[4][64 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = p.K, KK = K * K;
  for (int64_t n = (int64_t)blockIdx.x * 4 + wave; n < p.B * p.T; n += (int64_t)gridDim.x * 4) {
    const int64_t b = n / p.T;
    const int t = (int)(n - b * p.T);
    const float* u = p.u + b * (int64_t)p.U * p.T + (int64_t)t * p.u_st;
    for (int h = lane; h < p.TH; h += 64) {
      float v = p.b1[h];
      for (int c = 0; c < p.U; ++c) v = fmaf(p.W1[(int64_t)h * p.U + c], u[(int64_t)c * p.u_sc], v);
      hS[wave][h] = relu_f(v);
    }
    __builtin_amdgcn_wave_barrier();
    for (int ij = lane; ij < KK; ij += 64) {
      float z = p.b2[ij];
      const float* w2 = p.W2 + (int64_t)ij * p.TH;
      for (int h = 0; h < p.TH; ++h) z = fmaf(w2[h], hS[wave][h], z);
      zS[wave][ij] = z;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < K) {
      const float* zr = &zS[wave][lane * K];
      float m = -__builtin_inff();
      for (int j = 0; j < K; ++j) m = fmaxf(m, zr[j]);
      float s = 0.f;
      for (int j = 0; j < K; ++j) s += __expf(zr[j] - m);
      const float ls = m + __logf(s);
      for (int j = 0; j < K; ++j) p.log_A[n * KK + lane * K + j] = zr[j] - ls;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int launch_prior_fwd(const PriorArgs& p, hipStream_t s) {
  const int64_t N = p.B * p.T;
  if (N == 0) return VQHMM_OK;
  if (prior_mfma_supported(p) && (p.TH == 64 || p.TH == 128 || p.TH == 256)) return launch_prior_mfma(p, s);
  if (p.K <= 8 && p.U <= 8) {
    const dim3 grid((unsigned)cdiv(N, 256));
    if (p.K <= 4)
      prior_fwd_kernel<4, 8><<<grid, 256, 0, s>>>(p);
    else
      prior_fwd_kernel<8, 8><<<grid, 256, 0, s>>>(p);
  } else {
    if (p.K > 64 || p.TH > 1024) return VQHMM_EUNSUPPORTED;
    prior_fwd_wave_kernel<<<(unsigned)std::min<int64_t>(cdiv(N, 4), 4096), 256, 0, s>>>(p);
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
