// HMM recursions for K in (8, 32] states ("the API
// accepts any (B, T, K)"), e.g. a K = 32 model (BASELINE cfg3 dims).  Same
// contracts as hmm.hip (include/vqhmm.h, oracle/hmm_ref.py); the K <= 8 lane
// maps there hold a whole K x K step block in one wave, which stops at K = 8.
//
// Lane map: one sequence per wave.  K <= 32: lane l owns column j = l % 32 and
// the half h = l / 32 of the reduced axis (IH = 16 entries), one permlane32 swap
// joins the halves; K <= 16: column j = l % 16 and the quarter h = l / 16 (IH =
// 4), a permlane16 then a permlane32 join.  A step is IH independent adds per
// lane and one LDS broadcast of the new vector (no per-entry shuffles).
// The tables stream from HBM straight into registers one WHC-step chunk ahead
// of the chain (for a fixed reduced index the 32 lanes of a half read one
// contiguous row of log_A: coalesced).
//
// Viterbi: per step and column the argmax i is packed into a byte; 4 steps'
// bytes form one dword per column, stored as a (T/4, 32) uint32 table per
// sequence in the workspace.  The backtrace stages 256-step windows of it in
// LDS and chases them there.
// Forward-backward: wave 0 runs alpha, wave 1 beta of the same sequence; each
// step is a max-shifted log-sum-exp over the lane's IH terms, joined across the
// halves, with the previous vector's max and the step's max emission subtracted
// (their running sum is logZ's offset), so every stored value stays within a
// step's spread of 0.
// gamma = softmax(alpha + beta) over the workspace once both waves finish, one
// row per 32-lane half.
#include "kernels.h"
#include "prof.h"

namespace vqhmm {

namespace {

constexpr float WNEG_INF = -__builtin_inff();
constexpr int WHC = 4;    // steps per register chunk (prefetched one chunk ahead)
constexpr int WWIN = 256; // backtrace window (steps)

__device__ __forceinline__ int64_t wide_len(const int64_t* lengths, int64_t b, int T) {
  const int64_t L = lengths[b];
  return L <= 0 ? 0 : (L < T ? L : T);
}

// column orientation (alpha, Viterbi): a[s][ii] = A_t(i0 + ii, j), e[s] = em_t(j), t = t0 + s
// (clamped into [0, T), values past the chain's end are unused)
template <int IH, int W = WHC>
__device__ __forceinline__ void load_col_chunk(const float* __restrict__ A, const float* __restrict__ E, int K, int T,
                                               int t0, int j, int i0, float (&a)[W][IH], float (&e)[W]) {
#pragma unroll
  for (int s = 0; s < W; ++s) {
    const int t = min(t0 + s, T - 1);
    const float* At = A + (int64_t)t * K * K;
#pragma unroll
    for (int ii = 0; ii < IH; ++ii) {
      const int i = i0 + ii;
      a[s][ii] = (j < K && i < K) ? At[i * K + j] : WNEG_INF;
    }
    e[s] = j < K ? E[(int64_t)t * K + j] : 0.f;
  }
}

// row orientation (beta): a[s][jj] = A_t(i, j0 + jj), e[s] = em_t(i), t = t0 - s
// V4 (K % 4 == 0, 16-B aligned A): one 16-B load per 4 entries (a quad is wholly inside or outside the row);
// the scalar form's 32 lanes of a half each read a different row, 32 cache lines per instruction
template <int IH, int W = WHC, bool V4 = false>
__device__ __forceinline__ void load_row_chunk(const float* __restrict__ A, const float* __restrict__ E, int K, int T,
                                               int t0, int i, int j0, float (&a)[W][IH], float (&e)[W]) {
#pragma unroll
  for (int s = 0; s < W; ++s) {
    const int t = max(min(t0 - s, T - 1), 0);
    const float* Ar = A + (int64_t)t * K * K + (int64_t)(i < K ? i : 0) * K;
    if constexpr (V4) {
#pragma unroll
      for (int q = 0; q < IH / 4; ++q) {
        const int jc = j0 + 4 * q;
        const float4 v = (i < K && jc < K) ? *reinterpret_cast<const float4*>(Ar + jc)
                                           : make_float4(WNEG_INF, WNEG_INF, WNEG_INF, WNEG_INF);
        a[s][4 * q] = v.x; a[s][4 * q + 1] = v.y; a[s][4 * q + 2] = v.z; a[s][4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < IH; ++jj) {
        const int jc = j0 + jj;
        a[s][jj] = (i < K && jc < K) ? Ar[jc] : WNEG_INF;
      }
    }
    e[s] = i < K ? E[(int64_t)t * K + i] : 0.f;
  }
}

template <int IH>
__device__ __forceinline__ void read_half(const float* v32, int i0, float (&v)[IH]) {
#pragma unroll
  for (int q = 0; q < IH / 4; ++q) {
    const float4 f = *reinterpret_cast<const float4*>(v32 + i0 + 4 * q);
    v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
  }
}

// log-sum-exp of the lane's IH terms joined with the other half's (same result,
// bit for bit, in both halves: the join is evaluated half 0 first in each)
// NQ = 4 (K <= 16: 16 columns, the reduced axis in quarters): quarters 0+1 and 2+3 join first (xor16), then
// the pairs (xor32), the lower group first in every join, so all lanes of a column hold the same bits
template <int IH, int NQ = 2>
__device__ __forceinline__ float lse_join(const float (&x)[IH], int h) {
  float m = x[0];
#pragma unroll
  for (int k = 1; k < IH; ++k) m = fmaxf(m, x[k]);
  float s = 0.f;
  if (m != WNEG_INF) {
#pragma unroll
    for (int k = 0; k < IH; ++k) s += __expf(x[k] - m);
  }
  if constexpr (NQ == 4) {
    const float qm = xor16(m), qs = xor16(s);
    const bool up = h & 1;
    const float m0 = up ? qm : m, m1 = up ? m : qm, s0 = up ? qs : s, s1 = up ? s : qs;
    const float mq = fmaxf(m0, m1);
    s = mq == WNEG_INF ? 0.f : s0 * __expf(m0 - mq) + s1 * __expf(m1 - mq);
    m = mq;
    h >>= 1;
  }
  const float pm = xor32(m), ps = xor32(s);
  const float m0 = h ? pm : m, m1 = h ? m : pm, s0 = h ? ps : s, s1 = h ? s : ps;
  const float mm = fmaxf(m0, m1);
  if (mm == WNEG_INF) return WNEG_INF;
  const float tot = s0 * __expf(m0 - mm) + s1 * __expf(m1 - mm);
  return mm + __logf(tot);
}

}  // namespace

// --------------------------------------------------------------------- Viterbi
template <int IH, int NQ>
__global__ __launch_bounds__(64) void viterbi_wide_kernel(const float* __restrict__ log_pi,
                                                          const float* __restrict__ log_A,
                                                          const float* __restrict__ em,
                                                          const int64_t* __restrict__ lengths, int K, int T,
                                                          int32_t* __restrict__ path, float* __restrict__ score,
                                                          uint32_t* __restrict__ bp) {
  __shared__ __attribute__((aligned(16))) float dsh[2][32];
  __shared__ uint32_t win[WWIN / 4 * 32];
  __shared__ int pbuf[WWIN];
  // lane (h, j): column j of COLS = 64 / NQ, reduced-axis group h (NQ = 4 for K <= 16: every lane busy)
  constexpr int COLS = 64 / NQ;
  const int lane = threadIdx.x, j = lane % COLS, h = lane / COLS, i0 = h * IH;
  const int64_t b = blockIdx.x;
  const int L = (int)wide_len(lengths, b, T);
  int32_t* P = path + b * (int64_t)T;
  for (int t = L + lane; t < T; t += 64) P[t] = -1;
  if (L == 0) {
    if (lane == 0) score[b] = WNEG_INF;
    return;
  }
  const float* A = log_A + b * (int64_t)T * K * K;
  const float* E = em + b * (int64_t)T * K;
  uint32_t* BP = bp + b * (int64_t)cdiv(T, 4) * 32;

  float d = j < K ? log_pi[j] + E[j] : WNEG_INF;  // delta_0 = log_pi + e_0
  if (h == 0) dsh[0][j] = d;
  uint32_t bpw = 0;
  float ca[WHC][IH], ce[WHC], na[WHC][IH], ne[WHC];
  if (L > 1) load_col_chunk<IH>(A, E, K, T, 1, j, i0, ca, ce);
  for (int t0 = 1; t0 < L; t0 += WHC) {
    if (t0 + WHC < L) load_col_chunk<IH>(A, E, K, T, t0 + WHC, j, i0, na, ne);
#pragma unroll
    for (int s = 0; s < WHC; ++s) {
      const int t = t0 + s;
      if (t >= L) break;
      float dv[IH];
      read_half<IH>(dsh[(t - 1) & 1], i0, dv);
      // first max over the half (i ascending, strict '>': ties keep the lowest i)
      float m = dv[0] + ca[s][0];
      int arg = i0;
#pragma unroll
      for (int ii = 1; ii < IH; ++ii) {
        const float v = dv[ii] + ca[s][ii];
        if (v > m) { m = v; arg = i0 + ii; }
      }
      // join the groups, the lower one first (strict '>': its first max wins ties): quarters 0+1 and 2+3
      // (permlane16), then the pairs (permlane32); every lane of a column ends with the same (max, arg)
      int hh = h;
      if constexpr (NQ == 4) {
        const float qm = xor16(m);
        const int qa = xor16(arg);
        const bool hi = hh & 1;
        const float q0 = hi ? qm : m, q1 = hi ? m : qm;
        const int b0 = hi ? qa : arg, b1 = hi ? arg : qa;
        const bool upq = q1 > q0;
        m = upq ? q1 : q0;
        arg = upq ? b1 : b0;
        hh >>= 1;
      }
      const float pm = xor32(m);
      const int pa = xor32(arg);
      const float m0 = hh ? pm : m, m1 = hh ? m : pm;
      const int a0 = hh ? pa : arg, a1 = hh ? arg : pa;
      const bool up = m1 > m0;
      d = (up ? m1 : m0) + ce[s];
      bpw |= (uint32_t)(up ? a1 : a0) << (8 * (t & 3));
      if ((t & 3) == 3 || t == L - 1) {
        if (h == 0) BP[(t >> 2) * 32 + j] = bpw;
        bpw = 0;
      }
      if (h == 0) dsh[t & 1][j] = j < K ? d : WNEG_INF;
    }
#pragma unroll
    for (int s = 0; s < WHC; ++s) {
      ce[s] = ne[s];
#pragma unroll
      for (int ii = 0; ii < IH; ++ii) ca[s][ii] = na[s][ii];
    }
  }
  // last state: first argmax over j (lanes of one half hold d_{L-1}[j])
  float best = j < K ? d : WNEG_INF;
  int arg = j;
#pragma unroll
  for (int o = 1; o < COLS; o <<= 1) {
    const float ov = __shfl_xor(best, o);
    const int oa = __shfl_xor(arg, o);
    if (ov > best || (ov == best && oa < arg)) { best = ov; arg = oa; }
  }
  if (lane == 0) score[b] = best;

  // backtrace through 256-step windows of the byte table, top down
  __builtin_amdgcn_s_waitcnt(0);
  __threadfence_block();
  int s = arg;  // state at the current step (lane 0 walks)
  for (int w0 = ((L - 1) / WWIN) * WWIN; w0 >= 0; w0 -= WWIN) {
    const int hi = min(w0 + WWIN, L) - 1;
    const int nq = (hi >> 2) - (w0 >> 2) + 1;
    __syncthreads();
    for (int k = lane; k < nq * 32; k += 64) win[k] = BP[(int64_t)(w0 >> 2) * 32 + k];
    __syncthreads();
    if (lane == 0) {
      for (int t = hi; t >= w0; --t) {
        pbuf[t - w0] = s;
        if (t > 0) s = (int)((win[((t >> 2) - (w0 >> 2)) * 32 + s] >> (8 * (t & 3))) & 0xFFu);
      }
    }
    __syncthreads();
    for (int t = w0 + lane; t <= hi; t += 64) P[t] = pbuf[t - w0];
  }
}

// ------------------------------------------------------------ forward-backward
// ws: alpha [B][T][K] then beta [B][T][K] (both in natural log, per-step shifted)
// the max over the NQ lane groups of a column (exact: every lane gets the same value)
template <int NQ>
__device__ __forceinline__ float group_max(float m) {
  if constexpr (NQ == 4) m = fmaxf(m, xor16(m));
  return fmaxf(m, xor32(m));
}

template <int IH, int W, bool V4, int NQ>
__global__ __launch_bounds__(128) void fwdbwd_wide_kernel(const float* __restrict__ log_pi,
                                                          const float* __restrict__ log_A,
                                                          const float* __restrict__ em,
                                                          const int64_t* __restrict__ lengths, int64_t B, int K,
                                                          int T, float* __restrict__ gamma,
                                                          float* __restrict__ logZ, float* __restrict__ ws,
                                                          int dbg) {
  __shared__ __attribute__((aligned(16))) float vsh[2][2][32];  // [wave][parity][state]
  // lane (h, j): column j of COLS = 64 / NQ, reduced-axis group h (NQ = 4 for K <= 16: every lane busy)
  constexpr int COLS = 64 / NQ;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane % COLS, h = lane / COLS, i0 = h * IH;
  const int64_t b = blockIdx.x;
  const int L = (int)wide_len(lengths, b, T);
  const float* A = log_A + b * (int64_t)T * K * K;
  const float* E = em + b * (int64_t)T * K;
  float* AL = ws + b * (int64_t)T * K;
  float* BE = ws + (B + b) * (int64_t)T * K;
  float ca[W][IH], ce[W], na[W][IH], ne[W];

  if (L > 0 && wave == 0 && !(dbg & 4)) {
    // ---------------------------------------------------------------- alpha
    float e0 = j < K ? E[j] : WNEG_INF;
#pragma unroll
    for (int o = 1; o < COLS; o <<= 1) e0 = fmaxf(e0, __shfl_xor(e0, o));
    e0 = e0 == WNEG_INF ? 0.f : e0;
    float al = j < K ? log_pi[j] + (E[j] - e0) : WNEG_INF;
    if (h == 0) {
      vsh[0][0][j] = al;
      if (j < K) AL[j] = al;
    }
    double S = (double)e0;  // sum of the subtracted maxima (of alpha_{t-1} and of em_t)
    if (L > 1) load_col_chunk<IH, W>(A, E, K, T, 1, j, i0, ca, ce);
    for (int t0 = 1; t0 < L; t0 += W) {
      // emissions shifted by their max over the states, off the chain: em_t(j) - E_t
#pragma unroll
      for (int s = 0; s < W; ++s) {
        float em = j < K ? ce[s] : WNEG_INF;
#pragma unroll
        for (int o = 1; o < COLS; o <<= 1) em = fmaxf(em, __shfl_xor(em, o));
        em = em == WNEG_INF ? 0.f : em;
        ce[s] -= em;
        if (t0 + s < L) S += (double)em;
      }
      if (t0 + W < L) load_col_chunk<IH, W>(A, E, K, T, t0 + W, j, i0, na, ne);
#pragma unroll
      for (int s = 0; s < W; ++s) {
        const int t = t0 + s;
        if (t >= L) break;
        float v[IH];
        read_half<IH>(vsh[0][(t - 1) & 1], i0, v);
        float mh = v[0];
#pragma unroll
        for (int k = 1; k < IH; ++k) mh = fmaxf(mh, v[k]);
        float M = group_max<NQ>(mh);
        M = M == WNEG_INF ? 0.f : M;
        S += (double)M;
        float x[IH];
#pragma unroll
        for (int k = 0; k < IH; ++k) x[k] = (v[k] - M) + ca[s][k];
        const float lse = lse_join<IH, NQ>(x, h);
        al = j < K ? lse + ce[s] : WNEG_INF;
        if (h == 0) {
          vsh[0][t & 1][j] = al;
          if (j < K) AL[(int64_t)t * K + j] = al;
        }
      }
#pragma unroll
      for (int s = 0; s < W; ++s) {
        ce[s] = ne[s];
#pragma unroll
        for (int k = 0; k < IH; ++k) ca[s][k] = na[s][k];
      }
    }
    // logZ = S + LSE_j alpha_{L-1}(j)
    float mx = al;
#pragma unroll
    for (int o = 1; o < COLS; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float ex = (j < K && mx != WNEG_INF) ? __expf(al - mx) : 0.f;
#pragma unroll
    for (int o = 1; o < COLS; o <<= 1) ex += __shfl_xor(ex, o);
    if (lane == 0) logZ[b] = (float)(S + (double)mx + (double)__logf(ex));
  } else if (L > 0 && wave == 1 && !(dbg & 2)) {
    // ----------------------------------------------------------------- beta
    // lane's row state i = j; beta_{L-1} = 0
    float bv = j < K ? 0.f : WNEG_INF;
    if (h == 0 && j < K) BE[(int64_t)(L - 1) * K + j] = 0.f;
    if (L > 1) load_row_chunk<IH, W, V4>(A, E, K, T, L - 1, j, i0, ca, ce);
    for (int t0 = L - 1; t0 >= 1; t0 -= W) {  // data step t0 - s serves beta_{t0 - s - 1}
      if (t0 - W >= 1) load_row_chunk<IH, W, V4>(A, E, K, T, t0 - W, j, i0, na, ne);
#pragma unroll
      for (int s = 0; s < W; ++s) {
        const int td = t0 - s;
        if (td < 1) break;
        // w(j') = em_td(j') + beta_td(j') of every state j', through LDS
        if (h == 0) vsh[1][td & 1][j] = j < K ? ce[s] + bv : WNEG_INF;
        float w[IH];
        read_half<IH>(vsh[1][td & 1], i0, w);
        float nh = w[0];
#pragma unroll
        for (int k = 1; k < IH; ++k) nh = fmaxf(nh, w[k]);
        float N = group_max<NQ>(nh);
        N = N == WNEG_INF ? 0.f : N;
        float x[IH];
#pragma unroll
        for (int k = 0; k < IH; ++k) x[k] = ca[s][k] + (w[k] - N);
        const float lse = lse_join<IH, NQ>(x, h);
        bv = j < K ? lse : WNEG_INF;
        if (h == 0 && j < K) BE[(int64_t)(td - 1) * K + j] = bv;
      }
#pragma unroll
      for (int s = 0; s < W; ++s) {
        ce[s] = ne[s];
#pragma unroll
        for (int k = 0; k < IH; ++k) ca[s][k] = na[s][k];
      }
    }
  }
  if (L == 0 && threadIdx.x == 0) logZ[b] = __builtin_bit_cast(float, 0x7fc00000u);

  // ------------------------------------------------------------------- gamma
  __syncthreads();
  if (dbg & 1) return;  // timing experiment (profiling build, VQHMM_WIDE_DBG): no gamma pass
  // one row per 32-lane half (lane j = state j), four rows per pass: coalesced row reads and writes, the
  // softmax's max and sum as xor-shuffle trees inside the half
  const int gj = lane & 31, gh = lane >> 5;
  for (int t0 = 0; t0 < T; t0 += 4) {
    const int t = t0 + 2 * wave + gh;  // half-uniform
    if (t >= T) continue;
    float* g = gamma + (b * (int64_t)T + t) * K;
    if (t >= L) {
      if (gj < K) g[gj] = 0.f;
      continue;
    }
    const float x = gj < K ? AL[(int64_t)t * K + gj] + BE[(int64_t)t * K + gj] : WNEG_INF;
    float mx = x;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float e = (gj < K && mx != WNEG_INF) ? __expf(x - mx) : 0.f;
    float sm = e;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) sm += __shfl_xor(sm, o);
    if (gj < K) g[gj] = mx == WNEG_INF ? 0.f : e / sm;
  }
}

size_t viterbi_wide_ws_bytes(int64_t B, int64_t T) { return (size_t)B * (size_t)cdiv(T, 4) * 32 * 4; }

int launch_viterbi_wide(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                        int64_t T, int64_t K, int32_t* path, float* score, void* ws, hipStream_t s) {
  if (K <= 16)  // 16 columns x 4 quarters of 4 reduced entries
    viterbi_wide_kernel<4, 4><<<(unsigned)B, 64, 0, s>>>(log_pi, log_A, em, lengths, (int)K, (int)T, path, score,
                                                         (uint32_t*)ws);
  else  // 32 columns x 2 halves of 16
    viterbi_wide_kernel<16, 2><<<(unsigned)B, 64, 0, s>>>(log_pi, log_A, em, lengths, (int)K, (int)T, path, score,
                                                          (uint32_t*)ws);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_fwdbwd_wide(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                       int64_t T, int64_t K, float* gamma, float* logZ, float* ws, hipStream_t s) {
  // VQHMM_WIDE_DBG (profiling build; results invalid): 1 no gamma pass, 2 no beta chain, 4 no alpha chain
  static const int dbg = prof_env("VQHMM_WIDE_DBG");
  const bool v4 = K % 4 == 0 && (reinterpret_cast<uintptr_t>(log_A) & 15) == 0;
#define VQHMM_FBW(IHV, V4V, NQV)                                                                                  \
  fwdbwd_wide_kernel<IHV, WHC, V4V, NQV><<<(unsigned)B, 128, 0, s>>>(log_pi, log_A, em, lengths, B, (int)K, (int)T, gamma, \
                                                                logZ, ws, dbg)
  if (K <= 16) {  // 16 columns x 4 quarters of 4 reduced entries
    if (v4) VQHMM_FBW(4, true, 4);
    else VQHMM_FBW(4, false, 4);
  } else {  // 32 columns x 2 halves of 16
    if (v4) VQHMM_FBW(16, true, 2);
    else VQHMM_FBW(16, false, 2);
  }
#undef VQHMM_FBW
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
