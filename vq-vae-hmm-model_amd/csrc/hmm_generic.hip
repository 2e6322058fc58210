// HMM Viterbi and forward-backward for K > 32 states (the API takes any (B, T, K);
// hmm.hip packs K <= 8 into lane groups and hmm_wide.hip runs 8 < K <= 32 one sequence per wave).  Past 32
// states a step is a K x K contraction, so here one workgroup owns one sequence and thread j owns states
// j, j + 256, .. (S = ceil(K / 256) of them, K <= 256 S, S <= 16): the step reads log_A[t] as K coalesced
// rows (for fixed i the threads read consecutive j), the previous step's vector sits in LDS.  Semantics and
// contracts are the other kernels':
//   Viterbi  d_t[j] = (max_i d_{t-1}[i] + log_A[t][i][j]) + em[t][j] in fp32, i ascending, ties ->
//            lowest i; last state = first argmax; path -1 past the length, score -inf for length 0.
//            Bit-exact vs oracle/c/hmm_oracle.c (the same op order).  Backpointers: one byte per (t, j) in
//            the workspace for K <= 256, two above.
//   fwd-bwd  alpha / beta in log space renormalised every step (their log normalisers summed in fp64 give
//            logZ; they cancel in gamma = softmax_j(alpha_t + beta_t)); gamma 0 past the length, logZ NaN for
//            length 0, -inf for a zero-probability sequence.  Held to 1e-5 of the fp64 oracle like the other
//            kernels.
// Workspace: Viterbi B T K bytes (x2 above 256 states: backpointers); forward-backward B T K floats
// (normalised alpha).
#include "kernels.h"

namespace vqhmm {

namespace {
constexpr int HG_MAXS = 16;  // states per thread: K <= 4096

// block-wide max / sum of one value per thread (256 threads), result in every thread
__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
}  // namespace

template <int S, typename BP>
__global__ __launch_bounds__(256) void viterbi_generic_kernel(const float* __restrict__ log_pi,
                                                              const float* __restrict__ log_A,
                                                              const float* __restrict__ em,
                                                              const int64_t* __restrict__ lengths, int T, int K,
                                                              int32_t* __restrict__ path, float* __restrict__ score,
                                                              BP* __restrict__ bp) {
  __shared__ float dS[256 * S];
  __shared__ int sS;
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t L = lengths[b] < (int64_t)T ? lengths[b] : (int64_t)T;
  int32_t* pb = path + b * (int64_t)T;
  for (int t = tid; t < T; t += 256) pb[t] = -1;
  if (L <= 0) {
    if (tid == 0) score[b] = -__builtin_inff();
    return;
  }
  const float* e = em + b * (int64_t)T * K;
  const float* A = log_A + b * (int64_t)T * K * K;
  BP* bpb = bp + b * (int64_t)T * K;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int j = tid + 256 * s;
    if (j < K) dS[j] = log_pi[j] + e[j];
  }
  __syncthreads();
  for (int64_t t = 1; t < L; ++t) {
    const float* At = A + t * (int64_t)K * K;
    float best[S];
    int arg[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {  // S independent chains, each in the oracle's i order
      const int j = min(tid + 256 * s, K - 1);
      best[s] = dS[0] + At[j];
      arg[s] = 0;
    }
    for (int i = 1; i < K; ++i) {
      const float di = dS[i];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = min(tid + 256 * s, K - 1);
        const float v = di + At[(int64_t)i * K + j];
        if (v > best[s]) { best[s] = v; arg[s] = i; }
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = tid + 256 * s;
      if (j < K) {
        best[s] = best[s] + e[t * K + j];
        bpb[t * K + j] = (BP)arg[s];
      }
    }
    __syncthreads();  // every thread has read the previous vector
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = tid + 256 * s;
      if (j < K) dS[j] = best[s];
    }
    __syncthreads();
  }
  if (tid == 0) {
    int st = 0;
    for (int k = 1; k < K; ++k)
      if (dS[k] > dS[st]) st = k;
    score[b] = dS[st];
    sS = st;
  }
  __syncthreads();
  // backtrace: thread 0 follows the pointers (the workspace rows of this sequence were written by this
  // workgroup and are visible after the barrier above)
  if (tid == 0) {
    int st = sS;
    pb[L - 1] = st;
    for (int64_t t = L - 1; t > 0; --t) {
      st = bpb[t * K + st];
      pb[t - 1] = st;
    }
  }
}

// one state's online log-sum-exp step: x joins the running (m, s) of exp-sums
__device__ __forceinline__ void lse_push(float x, float& m, float& s) {
  if (x > m) {
    s = (m == -__builtin_inff() ? 0.f : s * __expf(m - x)) + 1.f;
    m = x;
  } else if (x > -__builtin_inff()) {
    s += __expf(x - m);
  }
}

// block max / sum of a thread's S values (reduced over s in order first)
template <int S>
__device__ __forceinline__ float block_max_s(const float (&v)[S], float* red) {
  float m = v[0];
#pragma unroll
  for (int s = 1; s < S; ++s) m = fmaxf(m, v[s]);
  return block_max(m, red);
}
template <int S>
__device__ __forceinline__ float block_sum_s(const float (&v)[S], float* red) {
  float m = v[0];
#pragma unroll
  for (int s = 1; s < S; ++s) m += v[s];
  return block_sum(m, red);
}

template <int S>
__global__ __launch_bounds__(256) void fwdbwd_generic_kernel(const float* __restrict__ log_pi,
                                                             const float* __restrict__ log_A,
                                                             const float* __restrict__ em,
                                                             const int64_t* __restrict__ lengths, int T, int K,
                                                             float* __restrict__ gamma, float* __restrict__ logZ,
                                                             float* __restrict__ alpha_ws) {
  __shared__ float vS[256 * S];  // alpha_{t-1} (forward), em_{t+1} + beta_{t+1} (backward)
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t L = lengths[b] < (int64_t)T ? lengths[b] : (int64_t)T;
  float* gb = gamma + b * (int64_t)T * K;
  for (int64_t i = (L > 0 ? L : 0) * K + tid; i < (int64_t)T * K; i += 256) gb[i] = 0.f;
  if (L <= 0) {
    if (tid == 0) logZ[b] = __builtin_nanf("");
    return;
  }
  const float* e = em + b * (int64_t)T * K;
  const float* A = log_A + b * (int64_t)T * K * K;
  float* al = alpha_ws + b * (int64_t)T * K;
  double lz = 0.0;
  constexpr float NINF = -__builtin_inff();
  // ---- forward: alpha_t(j) = LSE_i(alpha_{t-1}(i) + log_A[t][i][j]) + em[t][j], renormalised
  float v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int j = tid + 256 * s;
    v[s] = j < K ? log_pi[j] + e[j] : NINF;
  }
  for (int64_t t = 0; t < L; ++t) {
    if (t > 0) {
      const float* At = A + t * (int64_t)K * K;
      float m[S], sm[S];
#pragma unroll
      for (int s = 0; s < S; ++s) { m[s] = NINF; sm[s] = 0.f; }
      for (int i = 0; i < K; ++i) {
        const float vi = vS[i];
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int j = min(tid + 256 * s, K - 1);
          lse_push(vi + At[(int64_t)i * K + j], m[s], sm[s]);
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = tid + 256 * s;
        v[s] = j < K ? (m[s] == NINF ? m[s] : m[s] + __logf(sm[s])) + e[t * K + j] : NINF;
      }
    }
    const float mx = block_max_s<S>(v, red);
    float ex[S];
#pragma unroll
    for (int s = 0; s < S; ++s) ex[s] = tid + 256 * s < K ? __expf(v[s] - mx) : 0.f;
    const float n = mx == NINF ? mx : mx + __logf(block_sum_s<S>(ex, red));
    lz += (double)n;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (n != NINF) v[s] -= n;  // an impossible prefix stays -inf (logZ = -inf, as the fp64 oracle)
    __syncthreads();  // the previous vector is no longer read
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = tid + 256 * s;
      if (j < K) {
        vS[j] = v[s];
        al[t * K + j] = v[s];
      }
    }
    __syncthreads();
  }
  if (tid == 0) logZ[b] = (float)lz;
  // ---- backward: beta_t(i) = LSE_j(log_A[t+1][i][j] + em[t+1][j] + beta_{t+1}(j)), renormalised;
  // gamma_t = softmax_j(alpha_t + beta_t)
  float bt[S];  // beta_{L-1} = 0
#pragma unroll
  for (int s = 0; s < S; ++s) bt[s] = 0.f;
  for (int64_t t = L - 1; t >= 0; --t) {
    if (t < L - 1) {
      const float* At1 = A + (t + 1) * (int64_t)K * K;
      float m[S], sm[S];
#pragma unroll
      for (int s = 0; s < S; ++s) { m[s] = NINF; sm[s] = 0.f; }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = min(tid + 256 * s, K - 1);
        for (int jj = 0; jj < K; ++jj) lse_push(At1[(int64_t)j * K + jj] + vS[jj], m[s], sm[s]);
      }
      float bv[S];
#pragma unroll
      for (int s = 0; s < S; ++s) bv[s] = tid + 256 * s < K ? (m[s] == NINF ? m[s] : m[s] + __logf(sm[s])) : NINF;
      const float mx = block_max_s<S>(bv, red);
      float ex[S];
#pragma unroll
      for (int s = 0; s < S; ++s) ex[s] = tid + 256 * s < K ? __expf(bv[s] - mx) : 0.f;
      const float n = mx == NINF ? mx : mx + __logf(block_sum_s<S>(ex, red));
#pragma unroll
      for (int s = 0; s < S; ++s) bt[s] = n != NINF ? bv[s] - n : bv[s];
    }
    float g[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = tid + 256 * s;
      g[s] = j < K ? al[t * K + j] + bt[s] : NINF;
    }
    const float gm = block_max_s<S>(g, red);
    float ge[S];
#pragma unroll
    for (int s = 0; s < S; ++s) ge[s] = tid + 256 * s < K ? __expf(g[s] - gm) : 0.f;
    const float gs = block_sum_s<S>(ge, red);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = tid + 256 * s;
      if (j < K) gb[t * K + j] = ge[s] / gs;
    }
    __syncthreads();  // vS (em_{t+1} + beta_{t+1}) no longer read
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = tid + 256 * s;
      if (j < K) vS[j] = e[t * K + j] + bt[s];
    }
    __syncthreads();
  }
}

size_t hmm_generic_viterbi_ws_bytes(int64_t B, int64_t T, int64_t K) { return (size_t)B * T * K * (K > 256 ? 2 : 1); }
size_t hmm_generic_fwdbwd_ws_bytes(int64_t B, int64_t T, int64_t K) { return (size_t)B * T * K * sizeof(float); }
bool hmm_generic_supported(int64_t K) { return K >= 1 && K <= 256 * HG_MAXS; }

#define VQHMM_HG_S(X) \
  X(1) X(2) X(4) X(8) X(16)

int launch_viterbi_generic(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                           int64_t B, int64_t T, int64_t K, int32_t* path, float* score, void* ws, hipStream_t s) {
  if (!hmm_generic_supported(K) || T > INT32_MAX) return VQHMM_EUNSUPPORTED;
  if (B == 0) return VQHMM_OK;
  const int S = K <= 256 ? 1 : K <= 512 ? 2 : K <= 1024 ? 4 : K <= 2048 ? 8 : 16;
  if (S == 1)
    viterbi_generic_kernel<1, uint8_t><<<(unsigned)B, 256, 0, s>>>(log_pi, log_A, em, lengths, (int)T, (int)K, path,
                                                                   score, (uint8_t*)ws);
#define VQHMM_VG(SV)                                                                                          \
  else if (S == SV) viterbi_generic_kernel<SV, uint16_t><<<(unsigned)B, 256, 0, s>>>(log_pi, log_A, em, lengths, \
                                                                                     (int)T, (int)K, path, score, \
                                                                                     (uint16_t*)ws);
  VQHMM_VG(2) VQHMM_VG(4) VQHMM_VG(8) VQHMM_VG(16)
#undef VQHMM_VG
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_fwdbwd_generic(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                          int64_t B, int64_t T, int64_t K, float* gamma, float* logZ, void* ws, hipStream_t s) {
  if (!hmm_generic_supported(K) || T > INT32_MAX) return VQHMM_EUNSUPPORTED;
  if (B == 0) return VQHMM_OK;
  const int S = K <= 256 ? 1 : K <= 512 ? 2 : K <= 1024 ? 4 : K <= 2048 ? 8 : 16;
  switch (S) {
#define VQHMM_FG(SV)                                                                                              \
  case SV:                                                                                                        \
    fwdbwd_generic_kernel<SV><<<(unsigned)B, 256, 0, s>>>(log_pi, log_A, em, lengths, (int)T, (int)K, gamma, logZ, \
                                                          (float*)ws);                                            \
    break;
    VQHMM_HG_S(VQHMM_FG)
#undef VQHMM_FG
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}
#undef VQHMM_HG_S

}  // namespace vqhmm
