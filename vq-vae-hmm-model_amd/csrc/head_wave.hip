// Fused ELBO head with wave-independent windows (K <= 4, TH in {64, 128}, U <= 4, D <= 16):
// all of A4 + A8..A10 and their gradients (VQ_VAE_HMM_fixed.py:59-71 Prior MLP, :106-137 loss)
// per PCL row, the Prior MLP forward and backward on v_mfma_f32_16x16x4_f32.
//
// Every wave works alone on windows of 64 consecutive PCL rows (63 owned + 1 halo row whose
// log_A the last owned row needs for its t -> t+1 term); windows are dealt to waves across the
// whole grid, so no workgroup barrier sits between the phases of a window and the 2-4 waves
// of a SIMD drift into different phases: one wave's VALU phase B runs beside another's MFMA
// phases A / C.  Per window (lane p = row r0 + p in the row-wise phases):
//   L  the window's rows (prefetched in registers one window ahead) -> u' = [u, 1] in LDS
//   A  hid^T (TH x 16) = relu(W1' @ u'^T), lg^T (16 x 16) = W2 @ hid^T + b2, per 16-row block
//   B  lane = row: log_softmax -> log_A, recon NLL, entropy, init / transition terms, dq,
//      d log_A -> d lg (log_softmax backward); neighbours' q by lane shuffles, the next
//      row's log_A from the wave's LDS
//   C  hid, dhid = (dlg @ W2) * relu'(hid); gW2 += dlg^T @ hid, gW1' += dhid^T @ u' (db2 sums
//      dlg in phase B)
// Weight-gradient accumulators stay in registers across the wave's windows; the workgroup's
// 4 waves are summed in a fixed order at the end into one slab (deterministic).
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

namespace vqhmm {

namespace {
constexpr int LGS = 20;    // LDS row stride of lg / dlg (b128 reads of 16 rows hit distinct banks)

// NBW 16-row blocks per window: WROWS rows, the last one the halo
template <int HB, int NBW>
struct HwLds {
  static constexpr int WROWS = 16 * NBW;
  static constexpr int TH = HB * 16;
  static constexpr int LDW2 = TH + 4;  // W2S row stride: 4*LDW2 = 16 (mod 32) -> conflict-free
  float W2S[16 * LDW2];
  float W1S[TH * 8];  // W1' = [W1 | b1 | 0]  (TH x 8)
  struct Wave {
    float uS[WROWS * 8];
    float lgS[WROWS * LGS];
    float dlgS[WROWS * LGS];
  } wv[4];
  float lpS[4];
  unsigned long long cnt;
};

// one row's global inputs (raw loads from a clamped address; validity from r where used)
template <int DM>
struct HwRow {
  float4 u, q, lg;
  float par[2 * DM];
  float x[DM];
  int64_t L;
};

// row rc (clamped into [0, R)) of sequence b
template <int DM>
__device__ __forceinline__ void hw_load(const HeadArgs& a, int64_t rc, int b, HwRow<DM>& v) {
  v.L = a.lengths[b];
  v.u = *reinterpret_cast<const float4*>(a.u + rc * ld4(a.U));  // U > 4: channels 4.. are read in phase L
  v.q = *reinterpret_cast<const float4*>(a.q + rc * 4);
  v.lg = *reinterpret_cast<const float4*>(a.logits + rc * 4);
  const int ldp = ld4(2 * a.D), ldx = ld4(a.D);
#pragma unroll
  for (int c = 0; c < DM; ++c) {
    const int cc = min(c, a.D - 1);
    v.par[c] = a.par[rc * ldp + cc];
    v.par[DM + c] = a.par[rc * ldp + a.D + cc];
    v.x[c] = a.x[rc * ldx + min(c, ldx - 1)];
  }
}

__device__ __forceinline__ float f4(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
}  // namespace

template <int K, int HB, int DM, int NBW>
__global__ __launch_bounds__(256, 2) void elbo_head_wave_kernel(HeadArgs a) {
  constexpr int KK = K * K;
  constexpr int TH = HB * 16;
  constexpr int WROWS = 16 * NBW, WOWN = WROWS - 1;  // rows per window (incl. the halo row), owned rows
  using S = HwLds<HB, NBW>;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int U = a.U, D = a.D;
  const float Bn = loss_norm_batch(a.norm, a.B);
  const float cpri = -a.beta / Bn;  // d loss / d (init + trans)[b]
  const float cent = a.beta / Bn;   // d loss / d (sum q*log q)
  auto& W = sh.wv[wave];

  // windows dealt across the grid first: w = k * (4 * grid) + wave * grid + block
  const int64_t nwin = cdiv(a.R, WOWN);
  const int64_t stride = 4 * (int64_t)gridDim.x;
  // the slot rotates with the block so the waves that get one window more sit on different SIMDs
  int64_t w = (int64_t)((wave + blockIdx.x) & 3) * gridDim.x + blockIdx.x;
  // row inputs of window wl (lane p = row wl * WOWN + p, clamped; validity from r where used).  With
  // 1- or 2-block windows (small batches: a wave's chain, not the work, sets the time) the first
  // window's are issued here, in flight across the weight staging, and every later window's right after
  // the phase that last reads the current ones (B), in flight across phase C; 4-block windows have no
  // registers to spare for rows held across C (38-59 VGPRs of spill) and load at the window's start.
  constexpr bool PF_C = NBW <= 2;
  const unsigned Tp = (unsigned)a.T + 2u;
  HwRow<DM> cur;
  float qprev_cur = 0.f;
  auto load_win = [&](int64_t wl) {
    const int64_t rr = wl * WOWN + lane;
    const unsigned rc = (unsigned)(rr < a.R ? rr : a.R - 1);
    hw_load<DM>(a, rc, (int)(rc / Tp), cur);
    qprev_cur = a.q[(wl * WOWN - 1 < 0 ? 0 : wl * WOWN - 1) * 4 + (lane & 3)];  // lane k < K: q[r0 - 1][k]
  };
  if (PF_C && w < nwin) load_win(w);

  // ---- one-time: weights to LDS, log_pi, valid count
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < 16 * S::LDW2 && !(a.dbg & 16); i += 256) {
    const int ij = i / S::LDW2, h = i - ij * S::LDW2;
    sh.W2S[i] = (ij < KK && h < TH) ? a.W2[ij * TH + h] : 0.f;
  }
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < TH * 8; i += 256) {
    const int h = i >> 3, c = i & 7;
    sh.W1S[i] = c < U ? a.W1[h * U + c] : (c == U ? a.b1[h] : 0.f);
  }
  if (tid == 0) {
    float m = -__builtin_inff();
    for (int k = 0; k < K; ++k) m = fmaxf(m, a.log_prior[k]);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += __expf(a.log_prior[k] - m);
    const float l = m + __logf(s);
    for (int k = 0; k < 4; ++k) sh.lpS[k] = k < K ? a.log_prior[k] - l : 0.f;
    sh.cnt = a.norm ? (unsigned long long)a.norm[0] : a.cnt_in ? (unsigned long long)*a.cnt_in : 0ull;
  }
  f32x4 b2f;
#pragma unroll
  for (int v = 0; v < 4; ++v) b2f[v] = (4 * lg4 + v) < KK ? a.b2[4 * lg4 + v] : 0.f;
  __syncthreads();
  if (!a.norm && !a.cnt_in && !(a.dbg & 64)) {  // valid positions of the batch (mask.sum(), :120): one LDS atomic per wave
    unsigned c = 0;
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int64_t b = tid; b < a.B; b += 256) {
      const int64_t L = a.lengths[b];
      c += (unsigned)(L <= 0 ? 0 : (L < a.T ? L : a.T));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) atomicAdd(&sh.cnt, (unsigned long long)c);
  }
  __syncthreads();
  const float inv_n = 1.0f / fmaxf((float)(sh.cnt * (unsigned long long)D), 1.0f);
  float lp[K];
#pragma unroll
  for (int k = 0; k < K; ++k) lp[k] = sh.lpS[k];

  float s_rec = 0.f, s_ent = 0.f, s_tr = 0.f, s_init = 0.f;
  float q0acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) q0acc[k] = 0.f;
  f32x4 gW2[HB], gW1[HB];  // (ij x h) and (h x c') blocks, MFMA accumulators
  float db2v[KK];          // lane's (= row's) partial db2 (phase B)
#pragma unroll
  for (int i = 0; i < HB; ++i) {
    gW2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    gW1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int ij = 0; ij < KK; ++ij) db2v[ij] = 0.f;

  // ---- phase A on the window's NBW row blocks at once: lg^T -> lgS (NBW independent chains).
  // Software-pipelined over the hidden blocks: hb + 1's weight operands are read from LDS and its
  // hidden MFMAs issued behind hb's 16 output MFMAs (sched_barrier pins that order, so the
  // compiler cannot hoist every block's loads up front and spill); lg's chain order is unchanged.
  auto phase_a = [&]() {
    float ub0[NBW];
    f32x4 lg[NBW];
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      ub0[i] = W.uS[(i * 16 + l16) * 8 + lg4];
      lg[i] = b2f;
    }
    struct AW {
      float w1a;
      f32x4 b, w2v;
    };
    auto ldw = [&](int hb, AW& w) {  // u' = [u, 1]: the bias column is the accumulator's start
      // only u' columns c < U: column U holds the bias (1), which starts the accumulator instead
      // (with U < 4 the k = 4 contraction would otherwise add b1 a second time)
      w.w1a = lg4 < U ? sh.W1S[(hb * 16 + l16) * 8 + lg4] : 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) w.b[v] = sh.W1S[(hb * 16 + 4 * lg4 + v) * 8 + U];
      w.w2v = *reinterpret_cast<const f32x4*>(&sh.W2S[l16 * S::LDW2 + hb * 16 + 4 * lg4]);
    };
    auto hid = [&](const AW& w, f32x4 (&h)[NBW]) {
#pragma unroll
      for (int i = 0; i < NBW; ++i) h[i] = mfma16x16x4(w.w1a, ub0[i], w.b);
    };
    AW wv[2];
    f32x4 hc[2][NBW];
    ldw(0, wv[0]);
    hid(wv[0], hc[0]);
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
      const int cb = hb & 1;
      if (hb + 1 < HB) ldw(hb + 1, wv[cb ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v) hc[cb][i][v] = relu_f(hc[cb][i][v]);
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int i = 0; i < NBW; ++i) lg[i] = mfma16x16x4(wv[cb].w2v[v], hc[cb][i][v], lg[i]);
      if (hb + 1 < HB) hid(wv[cb ^ 1], hc[cb ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NBW; ++i) *reinterpret_cast<f32x4*>(&W.lgS[(i * 16 + l16) * LGS + 4 * lg4]) = lg[i];
  };

  // ---- phase C (MLP backward) on the window's NBW row blocks at once (NBW independent MFMA
  // chains per step hide the accumulator latency).  hid and dhid are produced in (rows x h)
  // layout, lane (lg4, l16) holding rows 4*lg4 + v of hidden unit hb*16 + l16; the
  // contractions over rows then map row 4*lg4 + s to MFMA step s, so register v = s of those
  // fragments IS the operand (no transposes).  db2 is summed in phase B instead.
  // Pipelined like phase A: hb + 1's hid / dhid MFMAs are issued behind hb's 8*NBW gradient MFMAs.
  auto phase_c = [&]() {
    constexpr int SD = (KK + 3) / 4;  // 4-wide contraction steps over ij that hold nonzero dlg
    float ua[NBW], dla[NBW][SD], dlt[NBW][4], ub[NBW][4];
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      ua[i] = lg4 < U ? W.uS[(i * 16 + l16) * 8 + lg4] : 0.f;                                      // u'[row l16][c lg4], c < U
#pragma unroll
      for (int s = 0; s < SD; ++s) dla[i][s] = W.dlgS[(i * 16 + l16) * LGS + 4 * s + lg4];         // dlg[row l16][ij 4s+lg4]
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        dlt[i][s] = W.dlgS[(i * 16 + 4 * lg4 + s) * LGS + l16];                                      // dlg[row 4lg4+s][ij l16]
        const float uv = W.uS[(i * 16 + 4 * lg4 + s) * 8 + (l16 & 7)];
        ub[i][s] = l16 < 8 ? uv : 0.f;                                                               // u'[row 4lg4+s][c' l16]
      }
    }
    struct CW {
      float w1, bb, w2b[SD];
    };
    auto ldw = [&](int hb, CW& w) {
      w.w1 = sh.W1S[(hb * 16 + l16) * 8 + lg4];                                                     // W1'[h][c lg4]
      w.bb = sh.W1S[(hb * 16 + l16) * 8 + U];                                                       // b1[h]
#pragma unroll
      for (int s = 0; s < SD; ++s) w.w2b[s] = sh.W2S[(4 * s + lg4) * S::LDW2 + hb * 16 + l16];    // W2[ij 4s+lg4][h]
    };
    auto fwd = [&](const CW& w, f32x4 (&h)[NBW], f32x4 (&dh)[NBW]) {
#pragma unroll
      for (int i = 0; i < NBW; ++i) {  // bias as the accumulator's start (u' = [u, 1], U <= 4)
        h[i] = mfma16x16x4(ua[i], w.w1, f32x4{w.bb, w.bb, w.bb, w.bb});
        dh[i] = mfma16x16x4(dla[i][0], w.w2b[0], f32x4{0.f, 0.f, 0.f, 0.f});
      }
#pragma unroll
      for (int s = 1; s < SD; ++s)  // ij >= K*K are zero: the steps past them are skipped
#pragma unroll
        for (int i = 0; i < NBW; ++i) dh[i] = mfma16x16x4(dla[i][s], w.w2b[s], dh[i]);
    };
    CW wv[2];
    f32x4 h[2][NBW], dh[2][NBW];
    ldw(0, wv[0]);
    fwd(wv[0], h[0], dh[0]);
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
      const int cb = hb & 1;
      if (hb + 1 < HB) ldw(hb + 1, wv[cb ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        f32x4 hr, dm;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          hr[v] = relu_f(h[cb][i][v]);
          dm[v] = h[cb][i][v] > 0.f ? dh[cb][i][v] : 0.f;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          gW2[hb] = mfma16x16x4(dlt[i][s], hr[s], gW2[hb]);   // (ij x h) += dlg^T . hid
          gW1[hb] = mfma16x16x4(dm[s], ub[i][s], gW1[hb]);    // (h x c') += dhid^T . u'
        }
      }
      if (hb + 1 < HB) fwd(wv[cb ^ 1], h[cb ^ 1], dh[cb ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  for (; w < nwin && !(a.dbg & 8); w += stride) {
    if (!PF_C) load_win(w);
    const int64_t r0 = w * WOWN;
    const int nown = (int)min<int64_t>(WOWN, a.R - r0);  // rows 0 .. nown-1 owned; row nown halo
    const int p = lane;
    const int64_t r = r0 + p;
    // (b, t) of the row in 32-bit arithmetic (R < 2^31, checked at launch)
    const unsigned rcl = (unsigned)(r < a.R ? r : a.R - 1);
    const int b = (int)(rcl / Tp);
    const int t = (int)(rcl - (unsigned)b * Tp) - 1;
    const bool valid = p <= nown && r < a.R && t >= 0 && t < a.T;
    const bool own = p < nown;
    const bool m = valid && t < cur.L;  // inside the sequence's length
    // ---------------- L: u' to LDS
    {
      float uv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) uv[c] = (valid && c < U && c < 4) ? f4(cur.u, c) : (c == U ? 1.f : 0.f);
      if (U > 4) {
#pragma unroll
        for (int c = 4; c < 8; ++c)
          if (valid && c < U) uv[c] = a.u[(r < a.R ? r : a.R - 1) * ld4(U) + c];
      }
      if (p < WROWS) {
        *reinterpret_cast<float4*>(&W.uS[p * 8]) = make_float4(uv[0], uv[1], uv[2], uv[3]);
        *reinterpret_cast<float4*>(&W.uS[p * 8 + 4]) = make_float4(uv[4], uv[5], uv[6], uv[7]);
      }
    }
    // ---------------- A: MLP forward (MFMA), lg^T -> lgS
    if (!(a.dbg & 1)) phase_a();
    if (!(a.dbg & 2)) {
    // ---------------- B: lane = row
    float qv[4], lgv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      qv[k] = (valid && k < K) ? f4(cur.q, k) : 0.f;
      lgv[k] = valid ? f4(cur.lg, k) : 0.f;
    }
    float la[KK];
    const int pw_ = p < WROWS ? p : WROWS - 1;  // lanes past the window mirror its last row, unused
    {
      float* lr = &W.lgS[pw_ * LGS];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        float mx = lr[i * K];
#pragma unroll
        for (int j = 1; j < K; ++j) mx = fmaxf(mx, lr[i * K + j]);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < K; ++j) s += __expf(lr[i * K + j] - mx);
        const float ls = mx + __logf(s);
#pragma unroll
        for (int j = 0; j < K; ++j) la[i * K + j] = lr[i * K + j] - ls;
      }
      if (p < WROWS)
#pragma unroll
        for (int ij = 0; ij < KK; ++ij) lr[ij] = la[ij];
    }
    // recon NLL (owned rows inside the length) and its gradient
#pragma unroll
    for (int c = 0; c < DM; ++c) {
      if (c >= D) break;
      float dmu = 0.f, dlv = 0.f;
      if (own && m) {
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
      if (a.need_grad && own) {
        a.dpar[r * ld4(2 * D) + c] = dmu;
        a.dpar[r * ld4(2 * D) + D + c] = dlv;
      }
    }
    if (a.need_grad && own)
      for (int c = 2 * D; c < ld4(2 * D); ++c) a.dpar[r * ld4(2 * D) + c] = 0.f;
    // entropy and its direct logits gradient
    {
      float mx = -__builtin_inff();
#pragma unroll
      for (int k = 0; k < K; ++k) mx = fmaxf(mx, lgv[k]);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) se += __expf(lgv[k] - mx);
      const float lse = mx + __logf(se);
      float f = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) f = fmaf(qv[k], lgv[k] - lse, f);
      if (own && m) s_ent -= f;
      if (a.need_grad && own) {
        f32x4 d4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < K; ++k) d4[k] = m ? cent * qv[k] * ((lgv[k] - lse) - f) : 0.f;
        *reinterpret_cast<f32x4*>(a.dlx + r * 4) = d4;
      }
    }
    const bool first = own && valid && t == 0;
    if (first) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        s_init = fmaf(qv[k], lp[k], s_init);
        q0acc[k] += qv[k];
      }
    }
    // neighbours: q of rows p - 1 and p + 1 (row r0 - 1 from the prefetch), pair weights
    const float wgt = (valid && t >= 1 && t < cur.L) ? 1.f : 0.f;  // pair (t-1, t) inside the length
    float qp[4], qn[4];
    {
      const int tprev = (int)((unsigned)(r0 > 0 ? r0 - 1 : 0) % Tp) - 1;
      const bool vprev = r0 > 0 && tprev >= 0 && tprev < a.T;  // row r0 - 1 is a time step
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float pk = __shfl(qprev_cur, k);
        const float up = __shfl_up(qv[k], 1);
        qp[k] = p == 0 ? ((vprev && k < K) ? pk : 0.f) : up;
        qn[k] = __shfl_down(qv[k], 1);
      }
    }
    const float wnx = __shfl_down(wgt, 1);
    // transitions (pair (t-1, t) of this row), dq, d log_A -> d lg
    {
      float* dl = &W.dlgS[pw_ * LGS];
      if (own) {
        const float* lan = &W.lgS[(p + 1) * LGS];  // row p + 1's log_A (written above by lane p + 1)
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
            tr = fmaf(qp[i] * qv[j], l, tr);
            dq[j] = fmaf(qp[i], l, dq[j]);
            dla[j] = cpri * wgt * qp[i] * qv[j];
            rs += dla[j];
          }
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const float d = dla[j] - __expf(la[i * K + j]) * rs;
            dl[i * K + j] = d;
            db2v[i * K + j] += d;
          }
        }
#pragma unroll
        for (int ij = KK; ij < 16; ++ij) dl[ij] = 0.f;
        s_tr += wgt * tr;
        if (a.need_grad) {
          f32x4 d4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < K; ++j) {
            float nx = 0.f;
#pragma unroll
            for (int jj = 0; jj < K; ++jj) nx = fmaf(qn[jj], lan[j * K + jj], nx);
            float v = cpri * (wgt * dq[j] + wnx * nx);
            if (valid && t == 0) v = fmaf(cpri, lp[j], v);
            d4[j] = valid ? v : 0.f;
          }
          *reinterpret_cast<f32x4*>(a.dqx + r * 4) = d4;
        }
      } else if (p < WROWS) {
#pragma unroll
        for (int ij = 0; ij < 16; ++ij) dl[ij] = 0.f;
      }
    }
    }
    // the next window's rows: B was the last reader of cur / qprev_cur
    if (PF_C && w + stride < nwin) load_win(w + stride);
    // ---------------- C: MLP backward (MFMA)
    if (a.need_grad && !(a.dbg & 4)) {
      phase_c();
    }
  }

  // ---------------- epilogue: loss partials, q0 / db2 sums, weight-gradient partials.  The
  // whole LDS is scratch now: every wave parks its accumulators side by side, one barrier, then
  // wave w adds hidden blocks [w HB/4, (w+1) HB/4) over the 4 waves in wave order (deterministic,
  // the order wave 0 alone used) and writes that part of the workgroup's slab.
  if (a.dbg & 32) return;
  constexpr int NV = 8 * HB;  // accumulator floats per lane: gW2 (4 HB) + gW1 (4 HB)
  constexpr int HBW = HB / 4;  // hidden blocks per wave in the slab write
  float* xbuf = reinterpret_cast<float*>(smem4);
  double* pw = reinterpret_cast<double*>(xbuf + 4 * NV * 64);  // [4 waves][4] loss partials
  float* qw = reinterpret_cast<float*>(pw + 16);                // [4 waves][4] q0 sums
  float* bw = qw + 16;                                          // [4 waves][16] db2 sums
  double dsum[4] = {(double)s_rec, (double)s_init, (double)s_tr, (double)s_ent};
  if (!(a.dbg & 128)) {
#pragma unroll
    for (int k = 0; k < 4; ++k) dsum[k] = wave_sum_dpp(dsum[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) q0acc[k] = wave_sum_dpp(q0acc[k]);
#pragma unroll
    for (int ij = 0; ij < KK; ++ij) db2v[ij] = wave_sum_dpp(db2v[ij]);
  }
  lds_barrier();  // every wave is past its windows: W2S / W1S / wv[] are free (stores stay in flight)
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) pw[wave * 4 + k] = dsum[k];
#pragma unroll
    for (int k = 0; k < K; ++k) qw[wave * 4 + k] = q0acc[k];
#pragma unroll
    for (int ij = 0; ij < KK; ++ij) bw[wave * 16 + ij] = db2v[ij];
  }
  if (a.need_grad) {
    float* xb = xbuf + wave * NV * 64;
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
#pragma unroll
      for (int v = 0; v < 4; ++v) xb[(hb * 4 + v) * 64 + lane] = gW2[hb][v];
#pragma unroll
      for (int v = 0; v < 4; ++v) xb[(4 * HB + hb * 4 + v) * 64 + lane] = gW1[hb][v];
    }
  }
  lds_barrier();
  if (a.dbg & 256) return;
  if (wave == 0) {
    if (lane < 4) a.part[blockIdx.x * 4 + lane] = ((pw[lane] + pw[4 + lane]) + pw[8 + lane]) + pw[12 + lane];
    if (a.need_grad) {
      if (lane < K) a.slab_q0[blockIdx.x * K + lane] = ((qw[lane] + qw[4 + lane]) + qw[8 + lane]) + qw[12 + lane];
      if (lane < KK)
        a.slab_b2[(int64_t)blockIdx.x * KK + lane] = ((bw[lane] + bw[16 + lane]) + bw[32 + lane]) + bw[48 + lane];
    }
  }
  if (!a.need_grad) return;
  auto sum4 = [&](int slot) {
    const float* x = xbuf + slot * 64 + lane;
    return ((x[0] + x[NV * 64]) + x[2 * NV * 64]) + x[3 * NV * 64];
  };
  float* sW2 = a.slab_W2 + (int64_t)blockIdx.x * KK * TH;
  float* sW1 = a.slab_W1 + (int64_t)blockIdx.x * TH * U;
  float* sb1 = a.slab_b1 + (int64_t)blockIdx.x * TH;
#pragma unroll
  for (int k = 0; k < HBW; ++k) {
    const int hb = wave * HBW + k;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ij = 4 * lg4 + v;
      const float g2 = sum4(hb * 4 + v);
      if (ij < KK) sW2[ij * TH + hb * 16 + l16] = g2;
      // gW1' block hb: lane -> h = hb*16 + 4*lg4 + v, c' = l16 (c' == U is db1)
      const int h = hb * 16 + 4 * lg4 + v;
      const float g1 = sum4(4 * HB + hb * 4 + v);
      if (l16 < U) sW1[h * U + l16] = g1;
      else if (l16 == U) sb1[h] = g1;
    }
  }
}

// Blocks per window: 4 (63 owned rows) from ~500 sequences of T = 200 up, 2 (31) from ~160, else 1 (15
// owned rows): at small batches the per-window chain, not the work, sets the time, so shorter windows on
// more waves finish sooner.  VQHMM_HEAD_NBW=1|4 overrides (A/B).
static int head_wave_nbw(int64_t R) {
  static const int force = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_HEAD_NBW");
    return e ? atoi(e) : 0;
  }();
  if (force == 1 || force == 2 || force == 4) return force;
  // measured (step ms, NBW 1 / 2 / 4): B = 1024 0.489 / 0.478 / 0.473, B = 512 0.293 / 0.282 / 0.280,
  // B = 256 0.187 / 0.181 / 0.191, B = 128 0.136 / 0.139 / 0.139 (T = 200)
  return R >= 98304 ? 4 : R >= 32768 ? 2 : 1;
}

// workgroups (= weight-gradient slabs the tail reduces): up to 512 (2 per CU); VQHMM_HEAD_GRID caps it
// lower (tuning A/B, read once)
int head_wave_grid(int64_t R) {
  static const int cap = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_HEAD_GRID");
    const int v = e ? atoi(e) : 0;
    return v >= 64 && v <= 512 ? v : 512;
  }();
  const int64_t nwin = cdiv(R, 16 * head_wave_nbw(R) - 1);
  return (int)(nwin < cap ? (nwin > 0 ? nwin : 1) : cap);
}

template <int NBW>
static size_t head_wave_lds(int HB) {
  const size_t ex = (size_t)4 * 8 * HB * 64 * 4 + 512;  // epilogue exchange buffer
  const size_t st = HB == 4 ? sizeof(HwLds<4, NBW>) : sizeof(HwLds<8, NBW>);
  return ex > st ? ex : st;
}

int launch_head_wave(const HeadArgs& a0, int grid, hipStream_t s) {
  static const int dbg = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_HEAD_DBG");
    return e ? atoi(e) : 0;
  }();
  HeadArgs a = a0;
  a.dbg = dbg;
  if (a.R >= (1ll << 31)) return VQHMM_EUNSUPPORTED;  // 32-bit row arithmetic
  const int nbw = head_wave_nbw(a.R);
#define VQHMM_HW(KV, HBV)                                                                              \
  {                                                                                                    \
    if (nbw == 4) {                                                                                    \
      const size_t lds = head_wave_lds<4>(HBV);                                                        \
      if (a.D <= 8) elbo_head_wave_kernel<KV, HBV, 8, 4><<<grid, 256, lds, s>>>(a);                   \
      else elbo_head_wave_kernel<KV, HBV, 16, 4><<<grid, 256, lds, s>>>(a);                           \
    } else if (nbw == 2) {                                                                             \
      const size_t lds = head_wave_lds<2>(HBV);                                                        \
      if (a.D <= 8) elbo_head_wave_kernel<KV, HBV, 8, 2><<<grid, 256, lds, s>>>(a);                   \
      else elbo_head_wave_kernel<KV, HBV, 16, 2><<<grid, 256, lds, s>>>(a);                           \
    } else {                                                                                           \
      const size_t lds = head_wave_lds<1>(HBV);                                                        \
      if (a.D <= 8) elbo_head_wave_kernel<KV, HBV, 8, 1><<<grid, 256, lds, s>>>(a);                   \
      else elbo_head_wave_kernel<KV, HBV, 16, 1><<<grid, 256, lds, s>>>(a);                           \
    }                                                                                                  \
  }
  const int HB = a.TH / 16;
  switch (a.K * 10 + HB) {
    case 14: VQHMM_HW(1, 4) break;
    case 18: VQHMM_HW(1, 8) break;
    case 24: VQHMM_HW(2, 4) break;
    case 28: VQHMM_HW(2, 8) break;
    case 34: VQHMM_HW(3, 4) break;
    case 38: VQHMM_HW(3, 8) break;
    case 44: VQHMM_HW(4, 4) break;
    case 48: VQHMM_HW(4, 8) break;
    default: return VQHMM_EUNSUPPORTED;
  }
#undef VQHMM_HW
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
