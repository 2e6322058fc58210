// HMM recursions over the Prior's tables.
//
// Semantic sources (no reference code): math.md:23-67 (pi, row-stochastic A_t
// conditioned on u_t), Prior.forward VQ_VAE_HMM_fixed.py:59-71 (log_pi,
// log_A (B,T,K,K)), transition indexing log_A[:, t] = t-1 -> t (:125-127).
// Exact contracts: include/vqhmm.h and oracle/hmm_ref.py.
//
// Lane mapping (K <= 8, KP = next pow2 >= K): a group of KP*KP lanes owns one
// sequence and holds the whole K x K transition block of a step, one (i, j)
// entry per lane, so the step's loads are one coalesced access and the
// reduction over the source state i is a butterfly across KP lanes.  The
// (i, j) <-> lane map ALTERNATES between steps ("outer": i = g / KP, j = g % KP;
// "inner": j = g / KP, i = g % KP): after reducing over i the result for state
// j sits in every lane whose j-coordinate is j, which is exactly the lane that
// needs it as its i-coordinate in the other map — no broadcast step.
// Sequences are independent: no inter-workgroup communication.
#include "kernels.h"

namespace vqhmm {

constexpr float NEG_INF = -__builtin_inff();

// butterfly over the KP lanes of the reduction axis (outer axis: stride KP; inner: stride 1)
template <int KP, bool OUTER>
__device__ __forceinline__ float allmax(float v) {
#pragma unroll
  for (int o = OUTER ? KP : 1; o < (OUTER ? KP * KP : KP); o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
template <int KP, bool OUTER>
__device__ __forceinline__ float allsum(float v) {
#pragma unroll
  for (int o = OUTER ? KP : 1; o < (OUTER ? KP * KP : KP); o <<= 1) v += __shfl_xor(v, o);
  return v;
}
// arg-max with the lowest index winning ties (associative, so any butterfly order
// yields the sequential "first maximum")
template <int KP, bool OUTER>
__device__ __forceinline__ void allargmax(float& v, int& a) {
#pragma unroll
  for (int o = OUTER ? KP : 1; o < (OUTER ? KP * KP : KP); o <<= 1) {
    const float ov = __shfl_xor(v, o);
    const int oa = __shfl_xor(a, o);
    if (ov > v || (ov == v && oa < a)) { v = ov; a = oa; }
  }
}
// log-sum-exp over the reduction axis; all -inf -> -inf
template <int KP, bool OUTER>
__device__ __forceinline__ float alllse(float v) {
  const float m = allmax<KP, OUTER>(v);
  if (m == NEG_INF) return NEG_INF;
  const float s = allsum<KP, OUTER>(__expf(v - m));
  return m + __logf(s);
}

// ------------------------------------------------------------------ Viterbi
// LDS: backpointers bp[seq_in_wave][t][j] (uint8) when they fit, else global ws.
template <int KP, bool BP_LDS>
__global__ __launch_bounds__(64) void viterbi_kernel(const float* __restrict__ log_pi, const float* __restrict__ log_A,
                                                     const float* __restrict__ em, const int64_t* __restrict__ lengths,
                                                     int64_t B, int T, int K, int32_t* __restrict__ path,
                                                     float* __restrict__ score, uint8_t* __restrict__ bp_ws) {
  constexpr int G = KP * KP, SPW = 64 / G;
  extern __shared__ uint8_t bps[];
  const int lane = threadIdx.x;
  const int grp = lane / G, g = lane % G;
  const int64_t b = (int64_t)blockIdx.x * SPW + grp;
  const bool live = b < B;
  const int64_t Lr = live ? lengths[b] : 0;
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  uint8_t* bp = BP_LDS ? bps + (size_t)grp * T * KP : bp_ws + (size_t)(live ? b : 0) * T * KP;
  const float* A = log_A + (size_t)(live ? b : 0) * T * K * K;
  const float* E = em + (size_t)(live ? b : 0) * T * K;
  // wave-uniform loop bound
  int Lmax = L;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) Lmax = max(Lmax, __shfl_xor(Lmax, o));

  // step 0 holds delta_0 indexed by the "inner" map's i = g % KP
  const int i0 = g % KP;
  float d = (L > 0 && i0 < K) ? log_pi[i0] + E[i0] : NEG_INF;
  for (int t = 1; t < Lmax; ++t) {
    const bool outer = (t & 1) == 0;
    const int i = outer ? g / KP : g % KP;
    const int j = outer ? g % KP : g / KP;
    const bool act = t < L;
    float a = (act && i < K && j < K) ? A[(size_t)t * K * K + i * K + j] : NEG_INF;
    float v = (i < K) ? d + a : NEG_INF;
    int arg = i;
    if (outer) allargmax<KP, true>(v, arg); else allargmax<KP, false>(v, arg);
    const float ej = (act && j < K) ? E[(size_t)t * K + j] : 0.f;
    if (act) {
      d = v + ej;
      if (i == 0 && j < K) bp[(size_t)t * KP + j] = (uint8_t)arg;
    }
  }
  // final argmax over the state axis the lanes currently hold
  const int tl = L - 1;  // last processed step; its map decides which axis holds the states
  const bool held_inner = (tl <= 0) || ((tl & 1) == 0);  // even step (or t=0): state = g % KP
  const int st = held_inner ? g % KP : g / KP;
  float v = (st < K) ? d : NEG_INF;
  int arg = st;
  if (held_inner) allargmax<KP, false>(v, arg); else allargmax<KP, true>(v, arg);
  if (BP_LDS) __syncthreads(); else __threadfence();
  // backtrace: one lane per sequence walks the backpointers; lanes stride the path writes
  int32_t* P = path + (size_t)(live ? b : 0) * T;
  if (live) {
    for (int t = L + g; t < T; t += G) P[t] = -1;
    if (g == 0) {
      if (L > 0) {
        score[b] = v;
        int s = arg;
        P[L - 1] = s;
        for (int t = L - 1; t > 0; --t) {
          s = bp[(size_t)t * KP + s];
          P[t - 1] = s;
        }
      } else {
        score[b] = NEG_INF;
      }
    }
  }
}

size_t viterbi_ws_bytes(int64_t B, int64_t T, int64_t K) {
  const int KP = K <= 2 ? 2 : K <= 4 ? 4 : 8;
  const size_t lds = (size_t)(64 / (KP * KP)) * T * KP;
  return lds <= 64 * 1024 ? 0 : (size_t)B * T * KP;
}

int launch_viterbi(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                   int64_t T, int64_t K, int32_t* path, float* score, void* ws, size_t ws_bytes, hipStream_t s) {
  if (B == 0) return VQHMM_OK;
  if (K < 1 || K > 8 || T < 1 || T > INT32_MAX) return VQHMM_EUNSUPPORTED;
  const int KP = K <= 2 ? 2 : K <= 4 ? 4 : 8;
  const int spw = 64 / (KP * KP);
  const size_t lds = (size_t)spw * T * KP;
  const bool in_lds = lds <= 64 * 1024;
  if (!in_lds && ws_bytes < (size_t)B * T * KP) return VQHMM_EWORKSPACE;
  const dim3 grid((unsigned)cdiv(B, spw));
  uint8_t* bw = (uint8_t*)ws;
#define VQHMM_VIT(KPV)                                                                                         \
  if (in_lds)                                                                                                  \
    viterbi_kernel<KPV, true><<<grid, 64, lds, s>>>(log_pi, log_A, em, lengths, B, (int)T, (int)K, path, score, \
                                                    bw);                                                       \
  else                                                                                                         \
    viterbi_kernel<KPV, false><<<grid, 64, 0, s>>>(log_pi, log_A, em, lengths, B, (int)T, (int)K, path, score, bw);
  if (KP == 2) { VQHMM_VIT(2) } else if (KP == 4) { VQHMM_VIT(4) } else { VQHMM_VIT(8) }
#undef VQHMM_VIT
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ---------------------------------------------------------- forward-backward
// Pass 1 (alpha, t ascending) stores the max-normalised alpha_t in ws and the
// accumulated normaliser; pass 2 (beta, t descending) forms gamma_t =
// softmax_j(alpha_t + beta_t) and writes it.  Both passes are in one launch
// (same wave, same sequence), so the alpha tile is re-read from L2.
template <int KP>
__global__ __launch_bounds__(64) void fwdbwd_kernel(const float* __restrict__ log_pi, const float* __restrict__ log_A,
                                                    const float* __restrict__ em, const int64_t* __restrict__ lengths,
                                                    int64_t B, int T, int K, float* __restrict__ gamma,
                                                    float* __restrict__ logZ, float* __restrict__ alpha_ws) {
  constexpr int G = KP * KP, SPW = 64 / G;
  const int lane = threadIdx.x;
  const int grp = lane / G, g = lane % G;
  const int64_t b = (int64_t)blockIdx.x * SPW + grp;
  const bool live = b < B;
  const int64_t Lr = live ? lengths[b] : 0;
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  const size_t bo = (size_t)(live ? b : 0);
  const float* A = log_A + bo * T * K * K;
  const float* E = em + bo * T * K;
  float* AL = alpha_ws + bo * T * K;
  float* GA = gamma + bo * T * K;
  int Lmax = L;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) Lmax = max(Lmax, __shfl_xor(Lmax, o));

  // ---- alpha pass.  After step t the lanes hold alpha_t(state) with state = g % KP
  // for even t (inner axis) and g / KP for odd t (outer axis).
  const int i0 = g % KP;
  float al = (L > 0 && i0 < K) ? log_pi[i0] + E[i0] : NEG_INF;
  float c = 0.f;  // sum of normalisers
  if (L > 0) {
    const float m = allmax<KP, false>(al);  // state on the inner axis at t = 0
    al -= m;
    c += m;
    if (g / KP == 0 && i0 < K) AL[i0] = al;
  }
  for (int t = 1; t < Lmax; ++t) {
    const bool outer = (t & 1) == 0;
    const int i = outer ? g / KP : g % KP;
    const int j = outer ? g % KP : g / KP;
    const bool act = t < L;
    const float a = (act && i < K && j < K) ? A[(size_t)t * K * K + i * K + j] : NEG_INF;
    float v = (i < K) ? al + a : NEG_INF;
    v = outer ? alllse<KP, true>(v) : alllse<KP, false>(v);
    v += (act && j < K) ? E[(size_t)t * K + j] : 0.f;
    if (j >= K) v = NEG_INF;
    // normalise over the states j (the other axis)
    const float m = outer ? allmax<KP, false>(v) : allmax<KP, true>(v);
    if (act) {
      al = v - m;
      c += m;
      if (i == 0 && j < K) AL[(size_t)t * K + j] = al;
    }
  }
  // logZ = c + LSE_j alpha_{L-1}(j): the states sit on the inner axis if L-1 is even
  {
    const int tl = L - 1;
    const bool inner = (tl <= 0) || ((tl & 1) == 0);
    const int st = inner ? g % KP : g / KP;
    float v = (st < K) ? al : NEG_INF;
    v = inner ? alllse<KP, false>(v) : alllse<KP, true>(v);
    if (live && g == 0) logZ[b] = L > 0 ? c + v : __builtin_nanf("");
  }
  __threadfence_block();
  // ---- beta pass (t descending); beta_{L-1} = 0.  The backward map mirrors the
  // forward one: at step t (computing beta_t from beta_{t+1}) the reduction is
  // over j; lanes hold beta_t(i) afterwards.  We use: step t even -> i = g / KP
  // (outer), j = g % KP, reduce over j = inner axis; t odd -> i = g % KP, j = g / KP,
  // reduce over the outer axis.  beta_{t+1} must then be held by state index j:
  // for even t, j = g % KP = inner — beta_{t+1} (t+1 odd) was produced as
  // beta(i = g % KP) held on the inner axis  (consistent); similarly for odd t.
  // Initial beta_{L-1} = 0 everywhere (any axis).
  for (int k = g; k < (T - L) * K; k += G)
    if (live) GA[(size_t)L * K + k] = 0.f;  // gamma beyond the length
  float be = 0.f;
  for (int t = Lmax - 1; t >= 0; --t) {
    const bool act = t < L;
    const bool even = (t & 1) == 0;
    const int i = even ? g / KP : g % KP;
    const int j = even ? g % KP : g / KP;
    float bnew = 0.f;
    if (t < L - 1) {
      // beta_t(i) = LSE_j (log_A[t+1, i, j] + e_{t+1}(j) + beta_{t+1}(j))
      const float a = (i < K && j < K) ? A[(size_t)(t + 1) * K * K + i * K + j] : NEG_INF;
      const float e = (j < K) ? E[(size_t)(t + 1) * K + j] : 0.f;
      float v = (j < K) ? a + e + be : NEG_INF;
      v = even ? alllse<KP, false>(v) : alllse<KP, true>(v);
      if (i >= K) v = NEG_INF;
      const float m = even ? allmax<KP, true>(v) : allmax<KP, false>(v);  // over states i
      bnew = v - m;
    } else {
      // butterflies stay inside a sequence's lane group, so groups may diverge here
      bnew = (i < K) ? 0.f : NEG_INF;
    }
    // gamma_t(i) = softmax_i(alpha_t(i) + beta_t(i)) over the state axis (outer if even)
    const float alv = (act && i < K) ? AL[(size_t)t * K + i] : NEG_INF;
    float sv = (act && i < K) ? alv + bnew : NEG_INF;
    const float mx = even ? allmax<KP, true>(sv) : allmax<KP, false>(sv);
    const float ex = (act && i < K && mx != NEG_INF) ? __expf(sv - mx) : 0.f;
    const float sm = even ? allsum<KP, true>(ex) : allsum<KP, false>(ex);
    if (act) {
      be = bnew;
      if (j == 0 && i < K) GA[(size_t)t * K + i] = ex / sm;
    }
  }
}

int launch_fwdbwd(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                  int64_t T, int64_t K, float* gamma, float* logZ, void* ws, size_t ws_bytes, hipStream_t s) {
  if (B == 0) return VQHMM_OK;
  if (K < 1 || K > 8 || T < 1 || T > INT32_MAX) return VQHMM_EUNSUPPORTED;
  if (ws_bytes < (size_t)B * T * K * sizeof(float)) return VQHMM_EWORKSPACE;
  const int KP = K <= 2 ? 2 : K <= 4 ? 4 : 8;
  const int spw = 64 / (KP * KP);
  const dim3 grid((unsigned)cdiv(B, spw));
  float* aw = (float*)ws;
  if (KP == 2)
    fwdbwd_kernel<2><<<grid, 64, 0, s>>>(log_pi, log_A, em, lengths, B, (int)T, (int)K, gamma, logZ, aw);
  else if (KP == 4)
    fwdbwd_kernel<4><<<grid, 64, 0, s>>>(log_pi, log_A, em, lengths, B, (int)T, (int)K, gamma, logZ, aw);
  else
    fwdbwd_kernel<8><<<grid, 64, 0, s>>>(log_pi, log_A, em, lengths, B, (int)T, (int)K, gamma, logZ, aw);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
