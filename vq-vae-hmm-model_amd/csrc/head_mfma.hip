// Fused ELBO head, MFMA version (K <= 4, TH in {64, 128}, U <= 7): the same
// math as head.hip (VQ_VAE_HMM_fixed.py:59-71 Prior MLP, :106-137 loss) with
// the Prior MLP forward and backward on v_mfma_f32_16x16x4_f32.
//
// Tile = 256 PCL rows (255 owned + 1 halo row whose log_A the last owned row
// needs for its t -> t+1 transition); 4 waves, wave w owns row blocks
// 4w..4w+3 of 16 rows.  Per 16-row block:
//   phase A  hid^T (TH x 16) = relu(W1' (TH x 8) @ u'^T (8 x 16))      u' = [u, 1], W1' = [W1, b1]
//            lg^T  (16 x 16) = W2 (16 x TH) @ hid^T + b2               (hid^T accumulator
//            fragments are the B operand as they stand: rows h = 4*(l>>4)+v)
//   phase B  VALU, thread per row: log_softmax -> log_A, recon NLL, entropy,
//            init/transition terms, dq, d log_A -> d lg (log_softmax backward)
//   phase C  hid, dhid = (dlg @ W2) * relu'(hid) in (rows x h) layout;
//            gW2' (16 x TH+16) += dlg^T @ [hid | 1]   (the ones column gives db2)
//            gW1' (TH x 16)   += dhid^T @ u'           (column U gives db1)
//            with row 4*(lane>>4) + s as contraction step s, the hid / dhid
//            accumulator registers are the operands directly (no transposes).
// Weight-gradient accumulators stay in registers across all tiles of the
// workgroup; the 4 waves are summed in fixed order at the end (deterministic).
#include <type_traits>

#include "kernels.h"

namespace vqhmm {

namespace {
constexpr int MP = 256;   // rows per tile (incl. halo)
constexpr int MOWN = 255; // owned rows

template <int K, int HB>
struct HeadLds {
  static constexpr int TH = HB * 16;
  static constexpr int LDW2 = TH + 4;   // W2S row stride: 4*LDW2 = 16 (mod 32) -> conflict-free
  float W2S[16 * LDW2];
  float W1S[TH * 8];      // W1' = [W1 | b1 | 0]  (TH x 8)
  float uS[MP * 8];
  float lgS[MP * 16];
  float dlgS[MP * 16];
  float qS[(MP + 2) * 4];
  int wS[MP + 2];
  float lpS[4];
  unsigned long long cnt;
};
}  // namespace

// Per-row global inputs of one tile, loaded one tile ahead into registers.
template <int K, int DM>
struct RowIn {
  float u[8];
  float q[4];
  float par[2 * DM];
  float x[DM];
  float lg[4];
  int64_t L;
};

template <int K, int DM>
__device__ __forceinline__ void load_row(const HeadArgs& a, int64_t r, RowIn<K, DM>& in) {
  // raw loads from clamped addresses of the PCL inputs; validity is re-derived
  // from r where the values are consumed (no select next to a load, so the
  // prefetch stays in flight)
  const int64_t rc = r < 0 ? 0 : (r >= a.R ? a.R - 1 : r);
  const int64_t b = rc / ((int64_t)a.T + 2);
  in.L = a.lengths[b];
  const int ldu = ld4(a.U), ldx = ld4(a.D), ldp = ld4(2 * a.D);
#pragma unroll
  for (int c = 0; c < 8; ++c) in.u[c] = a.u[rc * ldu + min(c, ldu - 1)];
  const float4 qv = *reinterpret_cast<const float4*>(a.q + rc * 4);
  const float4 lv = *reinterpret_cast<const float4*>(a.logits + rc * 4);
  in.q[0] = qv.x; in.q[1] = qv.y; in.q[2] = qv.z; in.q[3] = qv.w;
  in.lg[0] = lv.x; in.lg[1] = lv.y; in.lg[2] = lv.z; in.lg[3] = lv.w;
#pragma unroll
  for (int c = 0; c < DM; ++c) {
    const int cc = min(c, a.D - 1);
    in.par[c] = a.par[rc * ldp + cc];
    in.par[DM + c] = a.par[rc * ldp + a.D + cc];
    in.x[c] = a.x[rc * ldx + min(c, ldx - 1)];
  }
}

template <int K, int HB, int DM>
__global__ __launch_bounds__(256, 2) void elbo_head_mfma_kernel(HeadArgs a) {
  constexpr int KK = K * K;
  constexpr int TH = HB * 16;
  using S = HeadLds<K, HB>;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int U = a.U, D = a.D;
  const float Bn = loss_norm_batch(a.norm, a.B);
  const float cpri = -a.beta / Bn;  // d loss / d (init + trans)[b]
  const float cent = a.beta / Bn;   // d loss / d (sum q*log q)

  // ---- one-time: weights to LDS / registers, log_pi, valid count
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < 16 * S::LDW2; i += 256) {
    const int ij = i / S::LDW2, h = i - ij * S::LDW2;
    sh.W2S[i] = (ij < KK && h < TH) ? a.W2[ij * TH + h] : 0.f;
  }
  if (tid == 0) {
    float m = -__builtin_inff();
    for (int k = 0; k < K; ++k) m = fmaxf(m, a.log_prior[k]);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += __expf(a.log_prior[k] - m);
    const float l = m + __logf(s);
    for (int k = 0; k < K; ++k) sh.lpS[k] = a.log_prior[k] - l;
    sh.cnt = a.norm ? (unsigned long long)a.norm[0] : 0ull;
  }
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < TH * 8; i += 256) {
    const int h = i >> 3, c = i & 7;
    sh.W1S[i] = c < U ? a.W1[h * U + c] : (c == U ? a.b1[h] : 0.f);
  }
  // A fragments come from LDS: W1'[h = hb*16 + l16][c' = 4*ks + lg4] and, for lg^T,
  // W2[ij = l16][h = hb*16 + 4*lg4 + v] (one float4 per hidden block)
  f32x4 b2f;
#pragma unroll
  for (int v = 0; v < 4; ++v) b2f[v] = (4 * lg4 + v) < KK ? a.b2[4 * lg4 + v] : 0.f;
  __syncthreads();
  {
    unsigned long long c = 0;
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int64_t b = tid; !a.norm && b < a.B; b += 256) {
      const int64_t L = a.lengths[b];
      c += (unsigned long long)(L <= 0 ? 0 : (L < a.T ? L : a.T));
    }
    atomicAdd(&sh.cnt, c);
  }
  __syncthreads();
  const float inv_n = 1.0f / fmaxf((float)(sh.cnt * (unsigned long long)D), 1.0f);

  float s_rec = 0.f, s_ent = 0.f, s_tr = 0.f, s_init = 0.f;
  float q0acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) q0acc[k] = 0.f;
  f32x4 gW2[HB + 1], gW1[HB];
#pragma unroll
  for (int i = 0; i <= HB; ++i) gW2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < HB; ++i) gW1[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // This workgroup's rows: an equal share [rb, re) of all R rows, walked in
  // tiles of up to MOWN owned rows + 1 halo row (equal shares keep every CU
  // busy to the end; 16-row blocks past a short last tile are skipped).
  const int64_t rb = a.R * (int64_t)blockIdx.x / gridDim.x;
  const int64_t re = a.R * ((int64_t)blockIdx.x + 1) / gridDim.x;

  // ---- phase A on NP (1 or 2) row blocks of this wave at once: lg^T -> lgS
  auto phase_a = [&](auto np_tag, int blk0, int blk1) {
    constexpr int NP = decltype(np_tag)::value;
    const int p0[2] = {blk0 * 16, blk1 * 16};
    float ub0[NP], ub1[NP];
    f32x4 lg[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      ub0[i] = sh.uS[(p0[i] + l16) * 8 + lg4];
      ub1[i] = sh.uS[(p0[i] + l16) * 8 + 4 + lg4];
      lg[i] = b2f;
    }
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
      const float w1a = sh.W1S[(hb * 16 + l16) * 8 + lg4], w1b = sh.W1S[(hb * 16 + l16) * 8 + 4 + lg4];
      const f32x4 w2v = *reinterpret_cast<const f32x4*>(&sh.W2S[l16 * S::LDW2 + hb * 16 + 4 * lg4]);
      f32x4 h[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) h[i] = mfma16x16x4(w1a, ub0[i], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < NP; ++i) h[i] = mfma16x16x4(w1b, ub1[i], h[i]);
#pragma unroll
      for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v) h[i][v] = relu_f(h[i][v]);
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int i = 0; i < NP; ++i) lg[i] = mfma16x16x4(w2v[v], h[i][v], lg[i]);
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) *reinterpret_cast<f32x4*>(&sh.lgS[(p0[i] + l16) * 16 + 4 * lg4]) = lg[i];
  };

  // ---- phase C (MLP backward) on NP row blocks of this wave at once.  hid and
  // dhid are produced in (rows x h) layout, lane (lg4, l16) holding rows
  // 4*lg4 + v of hidden unit hb*16 + l16; the contractions over rows then map
  // row 4*lg4 + s to MFMA step s, so register v = s of those fragments IS the
  // operand (no transposes).
  auto phase_c = [&](auto np_tag, int blk0, int blk1) {
    constexpr int NP = decltype(np_tag)::value;
    constexpr int SD = (KK + 3) / 4;  // 4-wide contraction steps over ij that hold nonzero dlg
    const int p0[2] = {blk0 * 16, blk1 * 16};
    float ua[NP][2], dla[NP][4], dlt[NP][4], ub[NP][4];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
#pragma unroll
      for (int s = 0; s < 2; ++s) ua[i][s] = sh.uS[(p0[i] + l16) * 8 + 4 * s + lg4];       // u'[row l16][c 4s+lg4]
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        dla[i][s] = sh.dlgS[(p0[i] + l16) * 16 + 4 * s + lg4];                              // dlg[row l16][ij 4s+lg4]
        dlt[i][s] = sh.dlgS[(p0[i] + 4 * lg4 + s) * 16 + l16];                              // dlg[row 4lg4+s][ij l16]
        const float uv = sh.uS[(p0[i] + 4 * lg4 + s) * 8 + (l16 & 7)];
        ub[i][s] = l16 < 8 ? uv : 0.f;                                                      // u'[row 4lg4+s][c' l16]
      }
    }
    // db2: contraction of dlg^T with a ones column
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) gW2[HB] = mfma16x16x4(dlt[i][s], l16 == 0 ? 1.f : 0.f, gW2[HB]);
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
      float w1b[2], w2b[4];
#pragma unroll
      for (int s = 0; s < 2; ++s) w1b[s] = sh.W1S[(hb * 16 + l16) * 8 + 4 * s + lg4];        // W1'[h][c 4s+lg4]
#pragma unroll
      for (int s = 0; s < 4; ++s) w2b[s] = sh.W2S[(4 * s + lg4) * S::LDW2 + hb * 16 + l16];  // W2[ij 4s+lg4][h]
      f32x4 h[NP], dh[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        h[i] = mfma16x16x4(ua[i][0], w1b[0], f32x4{0.f, 0.f, 0.f, 0.f});
        dh[i] = mfma16x16x4(dla[i][0], w2b[0], f32x4{0.f, 0.f, 0.f, 0.f});
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) h[i] = mfma16x16x4(ua[i][1], w1b[1], h[i]);
#pragma unroll
      for (int s = 1; s < SD; ++s)  // ij >= K*K are zero: the steps past them add exact zeros
#pragma unroll
        for (int i = 0; i < NP; ++i) dh[i] = mfma16x16x4(dla[i][s], w2b[s], dh[i]);
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        f32x4 hr, dm;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          hr[v] = relu_f(h[i][v]);
          dm[v] = h[i][v] > 0.f ? dh[i][v] : 0.f;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          gW2[hb] = mfma16x16x4(dlt[i][s], hr[s], gW2[hb]);   // (ij x h) += dlg^T . hid
          gW1[hb] = mfma16x16x4(dm[s], ub[i][s], gW1[hb]);    // (h x c') += dhid^T . u'
        }
      }
    }
  };
  using One = std::integral_constant<int, 1>;
  using Two = std::integral_constant<int, 2>;
  // blocks of this wave in a tile: wave, wave + 4, wave + 8, wave + 12 (interleaved so a
  // short tile still spreads over the 4 waves), processed in pairs
  auto for_blocks = [&](int nblk, auto&& fn) {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int b0 = wave + 8 * pr, b1 = b0 + 4;
      if (b1 < nblk) fn(Two{}, b0, b1);
      else if (b0 < nblk) fn(One{}, b0, b0);
    }
  };
  auto for_blocks1 = [&](int nblk, auto&& fn) {
    for (int b0 = wave; b0 < nblk; b0 += 4) fn(One{}, b0, b0);
  };

  RowIn<K, DM> cur, nxt;
  load_row<K, DM>(a, rb + tid, cur);
  nxt = cur;
  for (int64_t r0 = rb; r0 < re; r0 += MOWN) {
    const int nown = (int)min<int64_t>(MOWN, re - r0);  // owned rows; row nown is the halo
    const int nblk = (nown + 16) / 16;                   // 16-row blocks holding rows 0..nown
    __syncthreads();
    // ---------------- L: stage this tile's rows (prefetched in registers)
    {
      const int64_t r = r0 + tid;
      int64_t b;
      int t;
      const bool valid = tid <= nown && row_bt(r, a.R, a.T, b, t);
      sh.wS[tid + 1] = (valid && t >= 1 && t < cur.L) ? 1 : 0;
#pragma unroll
      for (int c = 0; c < 8; ++c) sh.uS[tid * 8 + c] = (valid && c < U) ? cur.u[c] : (c == U ? 1.f : 0.f);
#pragma unroll
      for (int k = 0; k < 4; ++k) sh.qS[(tid + 1) * 4 + k] = (valid && k < K) ? cur.q[k] : 0.f;
      if (tid == 0) {
        const int64_t rp = r0 - 1;
        int64_t bp;
        int tp;
        const bool vp = row_bt(rp, a.R, a.T, bp, tp);
#pragma unroll
        for (int k = 0; k < 4; ++k) sh.qS[k] = (vp && k < K) ? a.q[rp * 4 + k] : 0.f;
        sh.wS[0] = (vp && tp >= 1 && tp < a.lengths[bp]) ? 1 : 0;
      }
    }
    __syncthreads();
    // ---------------- A: MLP forward (MFMA), lg^T -> lgS[p][ij]
    for_blocks(nblk, phase_a);
    __syncthreads();
    // ---------------- B1: log_softmax rows -> log_A (in place); recon, entropy, init
    {
      const int p = tid;
      const int64_t r = r0 + p;
      int64_t b;
      int t;
      const bool valid = row_bt(r, a.R, a.T, b, t);
      float* la = &sh.lgS[p * 16];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        float m = la[i * K];
#pragma unroll
        for (int j = 1; j < K; ++j) m = fmaxf(m, la[i * K + j]);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < K; ++j) s += __expf(la[i * K + j] - m);
        const float ls = m + __logf(s);
#pragma unroll
        for (int j = 0; j < K; ++j) la[i * K + j] -= ls;
      }
      if (p < nown) {
        const bool m = valid && t < cur.L;
#pragma unroll
        for (int c = 0; c < DM; ++c) {
          if (c >= D) break;
          float dmu = 0.f, dlv = 0.f;
          if (m) {
            const float mu = cur.par[c];
            const float lv = cur.par[DM + c];
            const float xv = cur.x[c];
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
        float lgv[K], qv[K];
        float mx = -__builtin_inff();
#pragma unroll
        for (int k = 0; k < K; ++k) {
          lgv[k] = valid ? cur.lg[k] : 0.f;
          qv[k] = valid ? cur.q[k] : 0.f;
          mx = fmaxf(mx, lgv[k]);
        }
        float se = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) se += __expf(lgv[k] - mx);
        const float lse = mx + __logf(se);
        float f = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) f = fmaf(qv[k], lgv[k] - lse, f);
        if (m) s_ent -= f;
        if (a.need_grad) {
          f32x4 d4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < K; ++k) d4[k] = m ? cent * qv[k] * ((lgv[k] - lse) - f) : 0.f;
          *reinterpret_cast<f32x4*>(a.dlx + r * 4) = d4;
        }
        if (valid && t == 0) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            s_init = fmaf(qv[k], sh.lpS[k], s_init);
            q0acc[k] += qv[k];
          }
        }
      }
    }
    __syncthreads();
    // ---------------- B2: transitions, dq, d lg (log_softmax backward) -> dlgS
    {
      const int p = tid;
      const int64_t r = r0 + p;
      float* dl = &sh.dlgS[p * 16];
      if (p < nown) {
        const float* qp = &sh.qS[p * 4];
        const float* qc = &sh.qS[(p + 1) * 4];
        const float* qn = &sh.qS[(p + 2) * 4];
        const float* la = &sh.lgS[p * 16];
        const float* lan = &sh.lgS[(p + 1) * 16];
        const float w = (float)sh.wS[p + 1];
        const float wn = (float)sh.wS[p + 2];
        float tr = 0.f;
        float dq[K];
#pragma unroll
        for (int j = 0; j < K; ++j) dq[j] = 0.f;
#pragma unroll
        for (int i = 0; i < K; ++i) {
          float rs = 0.f;
          float dla[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const float l = la[i * K + j];
            tr = fmaf(qp[i] * qc[j], l, tr);
            dq[j] = fmaf(qp[i], l, dq[j]);
            dla[j] = cpri * w * qp[i] * qc[j];
            rs += dla[j];
          }
#pragma unroll
          for (int j = 0; j < K; ++j) dl[i * K + j] = dla[j] - __expf(la[i * K + j]) * rs;
        }
#pragma unroll
        for (int ij = KK; ij < 16; ++ij) dl[ij] = 0.f;
        s_tr += w * tr;
        if (a.need_grad) {
          int64_t b;
          int t;
          const bool valid = row_bt(r, a.R, a.T, b, t);
          f32x4 d4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < K; ++j) {
            float nx = 0.f;
#pragma unroll
            for (int jj = 0; jj < K; ++jj) nx = fmaf(qn[jj], lan[j * K + jj], nx);
            float v = cpri * (w * dq[j] + wn * nx);
            if (valid && t == 0) v = fmaf(cpri, sh.lpS[j], v);
            d4[j] = valid ? v : 0.f;
          }
          *reinterpret_cast<f32x4*>(a.dqx + r * 4) = d4;
        }
      } else {
#pragma unroll
        for (int ij = 0; ij < 16; ++ij) dl[ij] = 0.f;
      }
    }
    if (r0 + MOWN < re) load_row<K, DM>(a, r0 + MOWN + tid, nxt);
    if (a.need_grad) {
      __syncthreads();
      // ---------------- C: MLP backward (MFMA)
      for_blocks1(nblk, phase_c);
    }
    cur = nxt;
  }

  // ---------------- epilogue: loss partials, q0 sums, weight-gradient partials
  __syncthreads();
  double* red = reinterpret_cast<double*>(sh.lgS);  // 4 x 256 doubles = 8 KB (lgS is 16 KB)
  red[0 * 256 + tid] = s_rec;
  red[1 * 256 + tid] = s_init;
  red[2 * 256 + tid] = s_tr;
  red[3 * 256 + tid] = s_ent;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st)
      for (int i = 0; i < 4; ++i) red[i * 256 + tid] += red[i * 256 + tid + st];
    __syncthreads();
  }
  if (tid < 4) a.part[blockIdx.x * 4 + tid] = red[tid * 256];
  if (!a.need_grad) return;
  float* qr = sh.dlgS;  // [K][256]
#pragma unroll
  for (int k = 0; k < K; ++k) qr[k * 256 + tid] = q0acc[k];
  __syncthreads();
  if (tid < K) {
    float s = 0.f;
    for (int i = 0; i < 256; ++i) s += qr[tid * 256 + i];
    a.slab_q0[blockIdx.x * K + tid] = s;
  }
  // weight grads: waves 1..3 add into wave 0 in order through LDS (uS region: 8 KB = 2048 floats)
  float* xch = sh.uS;
  constexpr int NV = (2 * HB + 1) * 4;  // floats per lane
  static_assert(NV * 64 <= MP * 8 + MP * 16, "exchange buffer");
  float* xbuf = sh.uS;  // uS (2048) followed by lgS (4096) are contiguous in HeadLds
  (void)xch;
  for (int w = 1; w < 4; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int hb = 0; hb <= HB; ++hb)
#pragma unroll
        for (int v = 0; v < 4; ++v) xbuf[(hb * 4 + v) * 64 + lane] = gW2[hb][v];
#pragma unroll
      for (int hb = 0; hb < HB; ++hb)
#pragma unroll
        for (int v = 0; v < 4; ++v) xbuf[((HB + 1 + hb) * 4 + v) * 64 + lane] = gW1[hb][v];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int hb = 0; hb <= HB; ++hb)
#pragma unroll
        for (int v = 0; v < 4; ++v) gW2[hb][v] += xbuf[(hb * 4 + v) * 64 + lane];
#pragma unroll
      for (int hb = 0; hb < HB; ++hb)
#pragma unroll
        for (int v = 0; v < 4; ++v) gW1[hb][v] += xbuf[((HB + 1 + hb) * 4 + v) * 64 + lane];
    }
  }
  if (wave == 0) {
    // gW2' block hb: lane -> ij = 4*lg4 + v, h = hb*16 + l16 (h == TH is db2)
    float* sW2 = a.slab_W2 + (int64_t)blockIdx.x * KK * TH;
    float* sb2 = a.slab_b2 + (int64_t)blockIdx.x * KK;
#pragma unroll
    for (int hb = 0; hb <= HB; ++hb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int ij = 4 * lg4 + v, h = hb * 16 + l16;
        if (ij < KK) {
          if (h < TH) sW2[ij * TH + h] = gW2[hb][v];
          else if (h == TH) sb2[ij] = gW2[hb][v];
        }
      }
    // gW1' block hb: lane -> h = hb*16 + 4*lg4 + v, c' = l16 (c' == U is db1)
    float* sW1 = a.slab_W1 + (int64_t)blockIdx.x * TH * U;
    float* sb1 = a.slab_b1 + (int64_t)blockIdx.x * TH;
#pragma unroll
    for (int hb = 0; hb < HB; ++hb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int h = hb * 16 + 4 * lg4 + v;
        if (l16 < U) sW1[h * U + l16] = gW1[hb][v];
        else if (l16 == U) sb1[h] = gW1[hb][v];
      }
  }
}

bool head_mfma_supported(const HeadArgs& a) {
  return a.K >= 1 && a.K <= 4 && a.U <= 7 && (a.TH == 64 || a.TH == 128) && a.D <= 16;
}

int launch_head_mfma(const HeadArgs& a, int grid, hipStream_t s) {
#define VQHMM_HM(KV, HBV)                                                                    \
  {                                                                                          \
    const size_t lds = sizeof(HeadLds<KV, HBV>);                                             \
    if (a.D <= 8)                                                                            \
      elbo_head_mfma_kernel<KV, HBV, 8><<<grid, 256, lds, s>>>(a);                           \
    else                                                                                     \
      elbo_head_mfma_kernel<KV, HBV, 16><<<grid, 256, lds, s>>>(a);                          \
  }
  const int HB = a.TH / 16;
  switch (a.K * 10 + HB) {
    case 14: VQHMM_HM(1, 4) break;
    case 18: VQHMM_HM(1, 8) break;
    case 24: VQHMM_HM(2, 4) break;
    case 28: VQHMM_HM(2, 8) break;
    case 34: VQHMM_HM(3, 4) break;
    case 38: VQHMM_HM(3, 8) break;
    case 44: VQHMM_HM(4, 4) break;
    case 48: VQHMM_HM(4, 8) break;
    default: return VQHMM_EUNSUPPORTED;
  }
#undef VQHMM_HM
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
