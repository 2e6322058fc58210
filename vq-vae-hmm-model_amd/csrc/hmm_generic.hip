// HMM Viterbi and forward-backward for 32 < K <= 256 states (the API takes
// any (B, T, K); hmm.hip packs K <= 8 into lane groups and hmm_wide.hip runs 8 < K <= 32 one
// sequence per wave).  Past 32 states a step is a K x K contraction, so here one workgroup owns one
// sequence and thread j owns state j (j + 256, ... for none: K <= 256): the step reads log_A[t] as K
// coalesced rows (for fixed i the threads read consecutive j), the previous step's vector sits in
// LDS.  Semantics and contracts are the other kernels':
//   Viterbi  d_t[j] = (max_i d_{t-1}[i] + log_A[t][i][j]) + em[t][j] in fp32, i ascending, ties ->
//            lowest i; last state = first argmax; path -1 past the length, score -inf for length 0.
//            Bit-exact vs oracle/c/hmm_oracle.c (the same op order).  Backpointers: one byte per
//            (t, j) in the workspace.
//   fwd-bwd  alpha / beta in log space renormalised every step (their log normalisers summed in
//            fp64 give logZ; they cancel in gamma = softmax_j(alpha_t + beta_t)); gamma 0 past the
//            length, logZ NaN for length 0.  Held to 1e-5 of the fp64 oracle like the other kernels.
// Workspace: Viterbi B T K bytes (backpointers); forward-backward B T K floats (normalised alpha).
#include "kernels.h"

namespace vqhmm {

namespace {
constexpr int HG_MAXK = 256;

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

__global__ __launch_bounds__(256) void viterbi_generic_kernel(const float* __restrict__ log_pi,
                                                              const float* __restrict__ log_A,
                                                              const float* __restrict__ em,
                                                              const int64_t* __restrict__ lengths, int T, int K,
                                                              int32_t* __restrict__ path, float* __restrict__ score,
                                                              uint8_t* __restrict__ bp) {
  __shared__ float dS[HG_MAXK];
  __shared__ int sS;
  const int64_t b = blockIdx.x;
  const int j = threadIdx.x;
  const int64_t L = lengths[b] < (int64_t)T ? lengths[b] : (int64_t)T;
  int32_t* pb = path + b * (int64_t)T;
  for (int t = j; t < T; t += 256) pb[t] = -1;
  if (L <= 0) {
    if (j == 0) score[b] = -__builtin_inff();
    return;
  }
  const float* e = em + b * (int64_t)T * K;
  const float* A = log_A + b * (int64_t)T * K * K;
  uint8_t* bpb = bp + b * (int64_t)T * K;
  if (j < K) dS[j] = log_pi[j] + e[j];
  __syncthreads();
  for (int64_t t = 1; t < L; ++t) {
    const float* At = A + t * (int64_t)K * K;
    float best = 0.f;
    int arg = 0;
    if (j < K) {
      best = dS[0] + At[j];
      for (int i = 1; i < K; ++i) {
        const float v = dS[i] + At[(int64_t)i * K + j];
        if (v > best) { best = v; arg = i; }
      }
      best = best + e[t * K + j];
      bpb[t * K + j] = (uint8_t)arg;
    }
    __syncthreads();  // every thread has read the previous vector
    if (j < K) dS[j] = best;
    __syncthreads();
  }
  if (j == 0) {
    int s = 0;
    for (int k = 1; k < K; ++k)
      if (dS[k] > dS[s]) s = k;
    score[b] = dS[s];
    sS = s;
  }
  __syncthreads();
  // backtrace: lane 0 follows the byte pointers (the workspace rows of this sequence were written
  // by this workgroup and are visible after the barrier above)
  if (j == 0) {
    int s = sS;
    pb[L - 1] = s;
    for (int64_t t = L - 1; t > 0; --t) {
      s = bpb[t * K + s];
      pb[t - 1] = s;
    }
  }
}

__global__ __launch_bounds__(256) void fwdbwd_generic_kernel(const float* __restrict__ log_pi,
                                                             const float* __restrict__ log_A,
                                                             const float* __restrict__ em,
                                                             const int64_t* __restrict__ lengths, int T, int K,
                                                             float* __restrict__ gamma, float* __restrict__ logZ,
                                                             float* __restrict__ alpha_ws) {
  __shared__ float vS[HG_MAXK];  // alpha_{t-1} (forward), em_{t+1} + beta_{t+1} (backward)
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const int j = threadIdx.x;
  const int64_t L = lengths[b] < (int64_t)T ? lengths[b] : (int64_t)T;
  float* gb = gamma + b * (int64_t)T * K;
  for (int64_t t = L > 0 ? L : 0; t < T; ++t)
    if (j < K) gb[t * K + j] = 0.f;
  if (L <= 0) {
    if (j == 0) logZ[b] = __builtin_nanf("");
    return;
  }
  const float* e = em + b * (int64_t)T * K;
  const float* A = log_A + b * (int64_t)T * K * K;
  float* al = alpha_ws + b * (int64_t)T * K;
  double lz = 0.0;
  // ---- forward: alpha_t(j) = LSE_i(alpha_{t-1}(i) + log_A[t][i][j]) + em[t][j], renormalised
  float v = j < K ? log_pi[j] + e[j] : -__builtin_inff();
  for (int64_t t = 0; t < L; ++t) {
    if (t > 0) {
      const float* At = A + t * (int64_t)K * K;
      float m = -__builtin_inff(), s = 0.f;  // online log-sum-exp over i
      if (j < K)
        for (int i = 0; i < K; ++i) {
          const float x = vS[i] + At[(int64_t)i * K + j];
          if (x > m) {
            s = (m == -__builtin_inff() ? 0.f : s * __expf(m - x)) + 1.f;
            m = x;
          } else if (x > -__builtin_inff()) {
            s += __expf(x - m);
          }
        }
      v = j < K ? (m == -__builtin_inff() ? m : m + __logf(s)) + e[t * K + j] : -__builtin_inff();
    }
    const float mx = block_max(v, red);
    const float n = (mx == -__builtin_inff() ? mx : mx + __logf(block_sum(j < K ? __expf(v - mx) : 0.f, red)));
    lz += (double)n;
    if (n != -__builtin_inff()) v -= n;  // an impossible prefix stays -inf (logZ = -inf, as the fp64 oracle)
    __syncthreads();  // the previous vector is no longer read
    if (j < K) {
      vS[j] = v;
      al[t * K + j] = v;
    }
    __syncthreads();
  }
  if (j == 0) logZ[b] = (float)lz;
  // ---- backward: beta_t(i) = LSE_j(log_A[t+1][i][j] + em[t+1][j] + beta_{t+1}(j)), renormalised;
  // gamma_t = softmax_j(alpha_t + beta_t)
  float bt = 0.f;  // beta_{L-1} = 0
  for (int64_t t = L - 1; t >= 0; --t) {
    if (t < L - 1) {
      const float* At1 = A + (t + 1) * (int64_t)K * K;
      float m = -__builtin_inff(), s = 0.f;
      if (j < K)
        for (int jj = 0; jj < K; ++jj) {
          const float x = At1[(int64_t)j * K + jj] + vS[jj];
          if (x > m) {
            s = (m == -__builtin_inff() ? 0.f : s * __expf(m - x)) + 1.f;
            m = x;
          } else if (x > -__builtin_inff()) {
            s += __expf(x - m);
          }
        }
      const float bv = j < K ? (m == -__builtin_inff() ? m : m + __logf(s)) : -__builtin_inff();
      const float mx = block_max(bv, red);
      const float n = (mx == -__builtin_inff() ? mx : mx + __logf(block_sum(j < K ? __expf(bv - mx) : 0.f, red)));
      bt = n != -__builtin_inff() ? bv - n : bv;
    }
    const float g = j < K ? al[t * K + j] + bt : -__builtin_inff();
    const float gm = block_max(g, red);
    const float ge = j < K ? __expf(g - gm) : 0.f;
    const float gs = block_sum(ge, red);
    if (j < K) gb[t * K + j] = ge / gs;
    __syncthreads();  // vS (em_{t+1} + beta_{t+1}) no longer read
    if (j < K) vS[j] = e[t * K + j] + bt;
    __syncthreads();
  }
}

size_t hmm_generic_viterbi_ws_bytes(int64_t B, int64_t T, int64_t K) { return (size_t)B * T * K; }
size_t hmm_generic_fwdbwd_ws_bytes(int64_t B, int64_t T, int64_t K) { return (size_t)B * T * K * sizeof(float); }

int launch_viterbi_generic(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                           int64_t B, int64_t T, int64_t K, int32_t* path, float* score, void* ws, hipStream_t s) {
  if (K < 1 || K > HG_MAXK || T > INT32_MAX) return VQHMM_EUNSUPPORTED;
  if (B == 0) return VQHMM_OK;
  viterbi_generic_kernel<<<(unsigned)B, 256, 0, s>>>(log_pi, log_A, em, lengths, (int)T, (int)K, path, score,
                                                    (uint8_t*)ws);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_fwdbwd_generic(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                          int64_t B, int64_t T, int64_t K, float* gamma, float* logZ, void* ws, hipStream_t s) {
  if (K < 1 || K > HG_MAXK || T > INT32_MAX) return VQHMM_EUNSUPPORTED;
  if (B == 0) return VQHMM_OK;
  fwdbwd_generic_kernel<<<(unsigned)B, 256, 0, s>>>(log_pi, log_A, em, lengths, (int)T, (int)K, gamma, logZ,
                                                   (float*)ws);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
