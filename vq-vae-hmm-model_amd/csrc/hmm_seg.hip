// Forward-backward, parallel in time.
//
// Semantics as hmm.hip (math.md:23-67; log_A[:, t] = t-1 -> t, VQ_VAE_HMM_fixed.py:125-127): per
// sequence b of length L, alpha_0 = log_pi + e_0, alpha_t(j) = LSE_i(alpha_{t-1}(i) + A_t(i, j)) + e_t(j),
// beta_{L-1} = 0, beta_{t-1}(i) = LSE_j(A_t(i, j) + e_t(j) + beta_t(j)), gamma_t = softmax(alpha_t + beta_t),
// logZ = LSE(alpha_{L-1}).
//
// The streaming / resident kernels of hmm.hip run each sequence as ONE chain of L serial steps (~140
// cycles a step): at the cfg4 shard (512 x 512, K = 8) that chain, not HBM, sets the time.  Here the
// sequence is cut into segments of SEG = 64 steps, one wave each, one workgroup per sequence:
//
//   P_t(i, j) = 2^((A_t(i, j) + e_t(j) - E_t) lg e),  E_t = max_j e_t(j)   (a per-step frame; linear domain)
//
//   phase 1  each wave loads its segment's table ONCE into 64 VGPRs (lane (r, c) holds entry (i, j) of
//            step t, the (i, j) <-> lane map alternating with t's parity as in hmm.hip) and forms the
//            segment's transfer matrix M_s = prod_t P_t on the matrix pipe: four 16-step chains per wave
//            as 16 blocks of v_mfma_f32_4x4x1f32, combined (M_0 M_1)(M_2 M_3) (layout at the code).
//   phase 2  one wave chains the S segment matrices forward for the alpha vector at every segment
//            boundary, another backward for beta (log2 domain, max-shifted LSE; S steps, not T; the vector
//            alternates lane axes step by step, so no LDS round trip sits in the chain).
//   phase 3  each wave reruns its segment's alpha and beta vector chains from those boundary vectors
//            on the tables still in its registers (the two chains interleaved, rescaled every 8 steps),
//            keeps both histories in LDS and writes gamma_t = alpha_t beta_t / sum for its 64 steps.
//
// HBM sees log_A and em once and gamma once (the algorithmic bytes); the serial chain is 16 + 2 matrix
// steps + S + 64 vector steps instead of L.  Range: a value that leaves [2^-96, 2^96] anywhere (a
// matrix entry relative to its row's last scale, a chain value relative to its last rescale) means
// something nearly vanished or exploded in fp32, as do -inf / NaN inputs (an exact 0 table entry, an
// all -inf emission row).  Then the whole sequence is recomputed by the exact path below (max-shifted
// natural-log recursions, renormalised every step, offsets in fp64, the workspace holding both
// directions): the tier fallback of hmm.hip, per sequence.
#include <type_traits>

#include "hmm_lanes.h"

namespace vqhmm {

constexpr int FBS_SEG = 64;       // time steps per segment (= per wave)
constexpr int FBS_MAXW = 16;      // segments per workgroup: T <= 1024
constexpr int FBS_WAVE_F = 1536;  // LDS floats per wave: es/hist_a [64][8] | hist_b [64][8] | P^T [2][4][8][8]
constexpr float FBS_LOG2E = 1.44269504088896341f;
constexpr double FBS_LN2 = 0.69314718055994531;
typedef float fbs_f4 __attribute__((ext_vector_type(4)));

// LDS of one workgroup of nw waves: the waves' regions, then the segment matrices (log2) [16][8][8], the
// boundary vectors alpha [17][8] and beta [17][8] (log2), the segments' frame sums (fp64) and flags.
__host__ __device__ constexpr size_t fbs_lds_bytes(int nw) {
  return (size_t)nw * FBS_WAVE_F * 4 + (1024 + 136 + 136) * 4 + FBS_MAXW * 8 + FBS_MAXW * 4;
}

__device__ __forceinline__ float fbs_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fbs_log2(float x) { return __builtin_amdgcn_logf(x); }
// c ? a : b with a computed unconditionally: left to itself the compiler turns the select into a branch
// around a's computation and sinks the step's table load into it, draining vmcnt there
__device__ __forceinline__ float fbs_pick(bool c, float a, float b) {
  asm volatile("" : "+v"(a));
  return c ? a : b;
}
__device__ __forceinline__ int fbs_bits(float x) { return __builtin_bit_cast(int, x); }
// a wave-uniform int in a VGPR: comparisons against it stay v_cmp / v_cndmask selects instead of
// scalar branches (which let the compiler sink a step's table load into a branch and drain vmcnt there)
__device__ __forceinline__ int fbs_vgpr(int x) {
  int v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
  return v;
}

// 8-lane all-reduces for the linear chains (values >= 0), as hmm_lanes.h's allred but (a) the max on bit
// patterns (v_max_i32: no NaN canonicalisation ops), (b) DPP without an "old" operand (folds into the add /
// max) and (c) the permlane swaps as plain asm, which the scheduler may interleave with another chain's
// (asm volatile pins every swap in program order: two chains in one wave then serialise)
__device__ __forceinline__ float2 fbs_pair16(float x) {
  float a = x, b = x;
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return make_float2(a, b);
}
__device__ __forceinline__ float2 fbs_pair32(float x) {
  float a = x, b = x;
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return make_float2(a, b);
}
template <int CTRL>
__device__ __forceinline__ float fbs_mdpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
template <bool INNER>
__device__ __forceinline__ float fbs_sum8(float v) {
  if constexpr (INNER) {
    v += fbs_mdpp<DPP_XOR1>(v);
    v += fbs_mdpp<DPP_XOR2>(v);
    v += fbs_mdpp<DPP_HALF_MIRROR>(v);
  } else {
    v += fbs_mdpp<DPP_ROR8>(v);
    const float2 a = fbs_pair16(v);
    v = a.x + a.y;
    const float2 c = fbs_pair32(v);
    v = c.x + c.y;
  }
  return v;
}
// two 8-lane sums over the outer axis at once (alpha's and beta's on even k): after the row_ror:8 adds, one
// 16-swap leaves a's row-pair sums in rows 0 / 2 and b's in 1 / 3, a 32-swap completes both, a last 16-swap
// spreads each over all rows (3 swaps for the two, 4 apart)
__device__ __forceinline__ void fbs_sum8_outer2(float a, float b, float& ya, float& yb) {
  a += fbs_mdpp<DPP_ROR8>(a);
  b += fbs_mdpp<DPP_ROR8>(b);
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));  // a = [a0 b0 a2 b2], b = [a1 b1 a3 b3]
  float c = a + b, d = c;
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(c), "+v"(d));  // c = [c0 c1 c0 c1], d = [c2 c3 c2 c3]
  float e = c + d, f = e;                                                 // [A B A B]
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(e), "+v"(f));  // e = [A A A A], f = [B B B B]
  ya = e;
  yb = f;
}
template <bool INNER>
__device__ __forceinline__ int fbs_maxb8(int v) {  // max of non-negative floats, on their bit patterns
  auto mx = [](int a, float b) { return max(a, __builtin_bit_cast(int, b)); };
  const float f = __builtin_bit_cast(float, v);
  if constexpr (INNER) {
    v = mx(v, fbs_mdpp<DPP_XOR1>(f));
    v = mx(v, fbs_mdpp<DPP_XOR2>(__builtin_bit_cast(float, v)));
    v = mx(v, fbs_mdpp<DPP_HALF_MIRROR>(__builtin_bit_cast(float, v)));
  } else {
    v = mx(v, fbs_mdpp<DPP_ROR8>(f));
    const float2 a = fbs_pair16(__builtin_bit_cast(float, v));
    v = max(__builtin_bit_cast(int, a.x), __builtin_bit_cast(int, a.y));
    const float2 c = fbs_pair32(__builtin_bit_cast(float, v));
    v = max(__builtin_bit_cast(int, c.x), __builtin_bit_cast(int, c.y));
  }
  return v;
}
// frexp exponent of the 8-lane max of x >= 0
template <bool INNER>
__device__ __forceinline__ int fbs_exp8(float x) {
  return __builtin_amdgcn_frexp_expf(__builtin_bit_cast(float, fbs_maxb8<INNER>(__builtin_bit_cast(int, x))));
}

// One workgroup per sequence, one wave per 64-step segment.  Steps that are not transitions of the
// sequence (t = 0, t >= L) carry the identity matrix, so every phase runs branch-free over its 64 steps:
// alpha / beta pass such a step unchanged and the product ignores it.
__global__ __launch_bounds__(1024) void fwdbwd_seg_kernel(const float* __restrict__ log_pi,
                                                          const float* __restrict__ log_A,
                                                          const float* __restrict__ em,
                                                          const int64_t* __restrict__ lengths, int64_t B, int T,
                                                          int K, float* __restrict__ gamma,
                                                          float* __restrict__ logZ, float* __restrict__ ws,
                                                          unsigned long long* __restrict__ prof) {
  constexpr int SEG = FBS_SEG;
  extern __shared__ float4 smem_fbs4[];
  float* sm = reinterpret_cast<float*>(smem_fbs4);
  const int nw = (int)(blockDim.x >> 6);
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)(threadIdx.x & 63), ra = lane >> 3, cb = lane & 7;
  const int64_t b = blockIdx.x;
  const int64_t Lr = lengths[b];
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  const int ts = w * SEG;  // first time step of this wave's segment (even: a step's parity is u's)
  float* gq = gamma + b * (int64_t)T * K;
  // profiling build only (VQHMM_FB_PROF=1, fast path): per wave s_memtime at the phase ends, [b][w][8]
  auto stamp = [&](int k) {
    if (prof && lane == 0) {
      const unsigned long long v = k == 0 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
      prof[((int64_t)b * FBS_MAXW + w) * 8 + k] = v;
      if (k == 7) prof[((int64_t)b * FBS_MAXW + w) * 8 + 1] = __builtin_amdgcn_s_memrealtime();
    }
  };
  if (prof && lane == 0) prof[((int64_t)b * FBS_MAXW + w) * 8 + 2] = __builtin_amdgcn_s_memtime();
  stamp(0);

  if (L == 0) {  // gamma = 0, logZ = NaN (hmm.hip's convention)
    for (int idx = (int)threadIdx.x; idx < T * K; idx += (int)blockDim.x) gq[idx] = 0.f;
    if (threadIdx.x == 0) logZ[b] = __builtin_bit_cast(float, 0x7fc00000u);
    return;
  }

  float* es = sm + w * FBS_WAVE_F;  // [64][8]: e_t(j) - E_t (natural); phase 3: alpha history
  float* hb = es + 512;             // [64][8]: beta history
  float* g_mlog = sm + nw * FBS_WAVE_F;  // [16][8][8] log2 M_s (row scale folded in)
  float* g_va = g_mlog + 1024;           // [17][8] alpha at segment boundaries (log2, framed)
  float* g_wb = g_va + 136;              // [17][8] beta at segment ends (log2)
  double* g_esum = reinterpret_cast<double*>(g_wb + 136);
  int* g_flag = reinterpret_cast<int*>(g_esum + FBS_MAXW);

  const float* Ab = log_A + b * (int64_t)T * K * K;
  const float* Eb = em + b * (int64_t)T * K;
  const int Kv = fbs_vgpr(K);
  const bool real = ra < Kv && cb < Kv;
  // the sequence's tables as buffers: loads past their end return 0 (steps past T are identity steps)
  const int stride = __builtin_amdgcn_readfirstlane(K * K * 4);  // bytes per step of log_A
  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, __builtin_amdgcn_readfirstlane(T * K * K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rE =
      __builtin_amdgcn_make_buffer_rsrc((void*)Eb, (short)0, __builtin_amdgcn_readfirstlane(T * K * 4), 0x00020000);
  // lane's entry of a step: (i, j) = (ra, cb) on even t, (cb, ra) on odd t
  const int voff0 = real ? (ra * K + cb) * 4 : 0, voff1 = real ? (cb * K + ra) * 4 : 0;
  auto tab_ld = [&](int u) -> float {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rA, (u & 1) ? voff1 : voff0,
                                                                         (ts + u) * stride, 0));
  };

  // ---------------------------------------------------------------- loads: em rows, then the table
  // lane l: the emission row of step ts + l
  const int tl = ts + lane;
  float er[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) er[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rE, tl * K * 4 + j * 4, 0, 0));
  float tab[SEG];
  // in phase 1's order (step s of the four chains: u = s, 16 + s, 32 + s, 48 + s); 8 + 48 loads in flight
  // (vmcnt counts to 63), the last 16 issued by phase 1's first four steps
  static_for<48>([&](auto ni) {
    constexpr int n = decltype(ni)::value, u = (n & 3) * 16 + (n >> 2);
    tab[u] = tab_ld(u);
  });
  float E = NEG_INF;
#pragma unroll
  for (int j = 0; j < 8; ++j) E = j < Kv ? fmaxf(E, er[j]) : E;
#pragma unroll
  for (int j = 0; j < 8; ++j) es[lane * 8 + j] = (er[j] - E) * FBS_LOG2E;  // (log2)
  // the frames of the sequence's steps in this segment (logZ = sum_t E_t + lg of the framed sums)
  const double esum = wave_sum_dpp((double)(tl < L ? E : 0.f));
  stamp(3);

  // ---------------------------------------------------------------- phase 1: M_s = prod_t P_t (matrix pipe)
  // Four chains per wave, chain q over the steps u = 16 q + s (s = 0..15), then (M_0 M_1)(M_2 M_3).  A chain
  // step is 8 v_mfma_f32_4x4x1f32 (16 blocks of 4 x 4 x 1): lane l = 16 q + 8 I + 4 J + x is row / column x
  // of block (q, I, J), and accumulator register i holds M(4 J + x, 4 I + i).  (M P) = sum_k M(:, k) P(k, :)
  // blockwise: MFMA n contracts k = n ^ 4 I (each block its own order), A = P(k, 4 I + x) from the chain's
  // P^T rows in LDS (written by the lanes of the table layout), B = M(4 J + x, k) = the lane's own register n
  // (n < 4) or its I-partner's (lane ^ 8, DPP row_ror:8) register n - 4.  Each step rescales every row by the
  // power of two of its max (row r's scale 2^cx on the two lanes holding it).
  const int q = lane >> 4, bI = (lane >> 3) & 1, bJ = (lane >> 2) & 1, bx = lane & 3;
  const int row = 4 * bJ + bx;
  const bool rowreal = row < Kv;
  fbs_f4 acc;
  int padm[4];  // or-masks: an entry outside K x K reads as 1.0 in the range checks
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = 4 * bI + i;
    acc[i] = (row == col && rowreal) ? 1.f : 0.f;
    padm[i] = (rowreal && col < Kv) ? 0 : fbs_bits(1.f);
  }
  const float ident = (ra == cb && ra < Kv) ? 1.f : 0.f;  // the table layout's identity entry
  float cx = 0.f;  // (a float sum: integer adds get reassociated into a tree holding every step's exponent)
  int lob = fbs_bits(1.f), hib = fbs_bits(1.f);  // range of the checked entries (bit patterns)
  const int ua = fbs_vgpr(max(0, min(SEG, L - ts)));  // steps u < ua are the sequence's (t < L)
  const int u_first = fbs_vgpr(w == 0 ? 1 : 0);      // (t = 0 is no transition)
  float* pbuf = es + 1024;                            // [2][4][8][8] the chains' P^T, double-buffered
  auto trans_of = [&](int u) { return (u < ua) & (u >= u_first); };
  auto rescale = [&]() {  // row max on the bit patterns (M >= 0: integer order = float order)
    const int m4 = max(max(fbs_bits(acc[0]), fbs_bits(acc[1])), max(fbs_bits(acc[2]), fbs_bits(acc[3])));
    const int m8 = max(m4, fbs_bits(fbs_mdpp<DPP_ROR8>(__builtin_bit_cast(float, m4))));
    const int e = __builtin_amdgcn_frexp_expf(__builtin_bit_cast(float, m8));
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_ldexpf(acc[i], -e);
    cx += (float)e;
  };
  auto checked = [&](int i, bool on) { return fbs_bits(acc[i]) | padm[i] | (on ? 0 : fbs_bits(1.f)); };
  auto check_lo = [&](bool on) {  // (a NaN or inf persists to the final check's hi)
    lob = min(lob, min(min(checked(0, on), checked(1, on)), min(checked(2, on), checked(3, on))));
    asm volatile("" : "+v"(lob));  // min is associative: unpinned, the 16 steps' values become a tree held to the end
  };
  auto check_lohi = [&](bool on) {
    check_lo(on);
    hib = max(hib, max(max(checked(0, on), checked(1, on)), max(checked(2, on), checked(3, on))));
  };
  auto mstep = [&](const float* pq) {  // pq[c * 8 + k] = P(k, c) of this lane's chain
    const float* pa = pq + (4 * bI + bx) * 8;
    const float4 a0 = *reinterpret_cast<const float4*>(pa + 4 * bI);
    const float4 a1 = *reinterpret_cast<const float4*>(pa + 4 - 4 * bI);
    float d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = fbs_mdpp<DPP_ROR8>(acc[i]);
    fbs_f4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a0.x, acc[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a0.y, acc[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a0.z, acc[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a0.w, acc[3], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a1.x, d[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a1.y, d[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a1.z, d[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a1.w, d[3], c, 0, 0, 0);
    acc = c;
  };
  static_for<SEG / 4>([&](auto si) {
    constexpr int s = decltype(si)::value, p = s & 1;
    const int i = p ? cb : ra, j = p ? ra : cb;
    float* pw = pbuf + (s & 1) * 256;
    static_for<4>([&](auto qi) {
      constexpr int qq = decltype(qi)::value, u = 16 * qq + s;
      const float P = fbs_exp2(fmaf(tab[u], FBS_LOG2E, es[u * 8 + j]));
      tab[u] = fbs_pick(real & trans_of(u), P, ident);  // not a transition: identity
      pw[qq * 64 + j * 8 + i] = tab[u];
    });
    if constexpr (s < 4) {
      static_for<4>([&](auto qi) {
        constexpr int u = 16 * decltype(qi)::value + 12 + s;
        tab[u] = tab_ld(u);
      });
    }
    if constexpr (s > 0) {
      rescale();
      check_lo(trans_of(16 * q + s - 1));
    }
    mstep(pw + q * 64);
  });
  rescale();
  check_lohi(trans_of(16 * q + 15));
  // combine: chain q + 1's matrix enters chain q's step as "P" = 2^(cx - cxm) M~ (cxm its largest real row
  // scale, added to chain q's rows); a product is checked when both factors hold a transition
  auto chain_max = [&](float v) {  // over the 16 lanes of a chain (rows: x and J; I repeats them)
    v = fmaxf(v, fbs_mdpp<DPP_XOR1>(v));
    v = fmaxf(v, fbs_mdpp<DPP_XOR2>(v));
    return fmaxf(v, fbs_mdpp<DPP_ROR4>(v));
  };
  auto has_t = [&](int qq) -> int { return ua > max(16 * qq, u_first); };
  auto feed = [&](float* pq, float cxm) {  // this chain's matrix as the "P" at pq (P^T layout)
#pragma unroll
    for (int i = 0; i < 4; ++i) pq[(4 * bI + i) * 8 + row] = __builtin_amdgcn_ldexpf(acc[i], (int)(cx - cxm));
  };
  {
    const float cxm = chain_max(rowreal ? cx : NEG_INF);
    if (q & 1) feed(pbuf + (q - 1) * 64, cxm);
    const float c1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cxm), 16));
    const float c3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cxm), 48));
    cx += q == 0 ? c1 : (q == 2 ? c3 : 0.f);
    mstep(pbuf + q * 64);
    rescale();
    check_lohi((int)((q & 1) == 0) & has_t(q) & has_t(q + 1));
  }
  {
    const float cxm = chain_max(rowreal ? cx : NEG_INF);
    if (q == 2) feed(pbuf + 256, cxm);
    cx += q == 0 ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cxm), 32)) : 0.f;
    mstep(pbuf + 256 + q * 64);
    rescale();
    check_lohi((int)(q == 0) & (has_t(0) | has_t(1)) & (has_t(2) | has_t(3)));
  }
  {
    // the rows' scales relative to the largest (exact small integers): lg M stays O(10) in fp32, the
    // common scale c0 goes to the fp64 frame sum
    const float c0 = chain_max(rowreal ? cx : NEG_INF);
    if (q == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = 4 * bI + i;
        const float ml = acc[i] > 0.f ? fbs_log2(acc[i]) + (cx - c0) : NEG_INF;
        g_mlog[w * 64 + row * 8 + col] = (rowreal && col < Kv) ? ml : NEG_INF;
      }
    }
    const bool bad = (int)(lob < fbs_bits(0x1p-96f)) | (int)(hib > fbs_bits(0x1p96f));
    const int anybad = __builtin_amdgcn_ballot_w64(bad) != 0;
    if (lane == 0) {
      g_flag[w] = anybad;
      g_esum[w] = esum + FBS_LN2 * (double)c0;
    }
  }
  stamp(4);
  __syncthreads();
  int flagged = 0;
  for (int s = 0; s < nw; ++s) flagged |= g_flag[s];

  // ---------------------------------------------------------------- phase 2: boundary vectors
  // Every segment's chain starts "at step -1" of the segment: segment 0 from alpha_0 (its step 0 is an
  // identity step), segment s from alpha at step 64 s - 1; beta from step 64 s + 63 (= beta_{L-1} past L).
  if (!flagged) {
    // The vectors alternate axes step by step (V on ra's axis, lanes (r, *) holding V(r), before an even
    // step; on cb's before an odd one), so each step reduces over the axis its input sits on and no LDS
    // round trip sits in the chain.  Each result is shifted by the max of its column maxima (reduced beside
    // the sum): V stays within [0, 3] at its max (a late segment's V would otherwise be ~-1e3 and its fp32
    // ulp a 1e-5 relative error in 2^V); the forward shifts are summed in fp64, beta's cancel.
    auto lse_step = [&](auto oddc, float v, float ml, float& sh) {  // LSE over the axis v sits on
      constexpr bool ODD = decltype(oddc)::value;
      const float x = v + ml;
      const float mx = allred<8, ODD>(x, OpMax{});
      const float ex = mx == NEG_INF ? 0.f : fbs_exp2(x - mx);
      sh = allred<8, !ODD>(mx, OpMax{});
      const float su = allred<8, ODD>(ex, OpAdd{});
      const float vn = mx == NEG_INF ? NEG_INF : mx + fbs_log2(su);
      return sh == NEG_INF ? vn : vn - sh;
    };
    // the two serial chains run while the workgroup's other waves wait at the barrier: raised priority,
    // so the co-resident workgroup's waves on the same SIMDs do not take their issue slots
    if (w <= 1) __builtin_amdgcn_s_setprio(3);
    if (w == 0) {
      // V_0(j) = lg alpha_0 (framed by E_0); V_{s+1}(c) = LSE_r(V_s(r) + lg M_s(r, c))
      const float v0 = cb < K ? fmaf(log_pi[cb], FBS_LOG2E, sm[cb]) : NEG_INF;  // sm = wave 0's es row 0
      if (lane < 8) g_va[lane] = v0;
      float v = ra < K ? fmaf(log_pi[ra], FBS_LOG2E, sm[ra]) : NEG_INF;  // V_0 on the ra axis
      double off = 0.0;
      auto fwd = [&](auto oddc, int s) {
        constexpr bool ODD = decltype(oddc)::value;
        float sh;
        v = lse_step(oddc, v, g_mlog[s * 64 + (ODD ? cb * 8 + ra : lane)], sh);  // M_s(r, c), r on v's axis
        off += sh == NEG_INF ? 0.0 : (double)sh;
        if ((ODD ? cb : ra) == 0) g_va[(s + 1) * 8 + (ODD ? ra : cb)] = v;
      };
      for (int s = 0; s < nw; s += 2) {
        fwd(std::false_type{}, s);
        if (s + 1 < nw) fwd(std::true_type{}, s + 1);
      }
      // logZ = ln 2 * (lg sum_j 2^V_S(j) + the offsets) + the frames; V_S on cb's axis for odd S
      const bool on_cb = nw & 1;
      const float vx = (on_cb ? cb : ra) < K ? v : NEG_INF;
      const float mx = on_cb ? allred<8, true>(vx, OpMax{}) : allred<8, false>(vx, OpMax{});
      const float ex = mx == NEG_INF ? 0.f : fbs_exp2(vx - mx);
      const float su = on_cb ? allred<8, true>(ex, OpAdd{}) : allred<8, false>(ex, OpAdd{});
      double fr = 0.0;
      for (int s = 0; s < nw; ++s) fr += g_esum[s];
      if (lane == 0) logZ[b] = (float)(FBS_LN2 * ((double)mx + (double)fbs_log2(su) + off) + fr);
    }
    if (w == (nw > 1 ? 1 : 0)) {
      // W_{S-1} = 0; W_{s-1}(r) = LSE_c(lg M_s(r, c) + W_s(c)) = beta at step 64 s - 1; W_{S-1} on cb's axis
      float v = cb < K ? 0.f : NEG_INF;
      if (lane < 8) g_wb[(nw - 1) * 8 + lane] = v;
      auto bwd = [&](auto oddc, int s) {
        constexpr bool ODD = decltype(oddc)::value;  // even: x(r = ra, c = cb), reduced over cb
        float sh;
        v = lse_step(std::integral_constant<bool, !ODD>{}, v, g_mlog[s * 64 + (ODD ? cb * 8 + ra : lane)], sh);
        if ((ODD ? ra : cb) == 0) g_wb[(s - 1) * 8 + (ODD ? cb : ra)] = v;
      };
      for (int s = nw - 1; s >= 1; s -= 2) {
        bwd(std::false_type{}, s);
        if (s - 1 >= 1) bwd(std::true_type{}, s - 1);
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
  __syncthreads();
  stamp(5);

  // ---------------------------------------------------------------- phase 3: the segment's chains + gamma
  if (!flagged) {
    float* ha = es;  // alpha history (the emission rows are no longer needed)
    // range checks on the bit patterns (values >= 0): an entry off the K axis or a step that is no
    // transition reads as 1.0 (or-mask), the min / max pinned per step (associative: left alone they become
    // a tree holding all 128 values)
    const int ubs = __builtin_amdgcn_readfirstlane(max(0, min(SEG, L - ts)));
    const int ufs = w == 0 ? 1 : 0;
    const int pm_ra = ra < Kv ? 0 : fbs_bits(1.f), pm_cb = cb < Kv ? 0 : fbs_bits(1.f);
    int lob = fbs_bits(1.f), hib = fbs_bits(1.f);
    auto masked = [&](float y, int pm, int u) {
      return fbs_bits(y) | pm | (((u < ubs) & (u >= ufs)) ? 0 : fbs_bits(1.f));
    };
    auto check2 = [&](int ta, int tb) {  // alpha's and beta's values of one k (v_min3 / v_max3)
      lob = min(lob, min(ta, tb));
      hib = max(hib, max(ta, tb));
      asm volatile("" : "+v"(lob), "+v"(hib));
    };
    // alpha starts on step 0's i axis (ra), beta on step 63's j axis (odd: ra)
    float xa, xb;
    {
      const float va = g_va[w * 8 + ra];
      const float ma = allred<8, false>(va, OpMax{});
      xa = ma == NEG_INF ? 0.f : fbs_exp2(va - ma);
      const float vb = g_wb[w * 8 + ra];
      const float mbx = allred<8, false>(vb, OpMax{});
      xb = mbx == NEG_INF ? 0.f : fbs_exp2(vb - mbx);
      hb[(SEG - 1) * 8 + ra] = xb;
    }
    static_for<SEG>([&](auto ki) {
      constexpr int k = decltype(ki)::value;
      // alpha step u = k reduces over i (even: ra, odd: cb), the result on the j axis; beta step 63 - k over
      // j (odd: ra, even: cb), the result on the i axis.  On even k both reduce over ra: one set of swaps
      float ya, yb;
      int ta;
      {
        float va = xa * tab[k], vb = tab[SEG - 1 - k] * xb;
        asm("" : "+v"(va), "+v"(vb));  // (else the product is folded into the first reduction step as an
                                        // fma, recomputing it beside a DPP move: 3 instructions for 2)
        if constexpr ((k & 1) == 0) fbs_sum8_outer2(va, vb, ya, yb);
        else {
          ya = fbs_sum8<true>(va);
          yb = fbs_sum8<true>(vb);
        }
      }
      {
        constexpr int u = k, p = u & 1;
        float y = ya;
        if constexpr (u % 8 == 4) {
          const int sx = fbs_exp8<p == 1>(xa);
          y = __builtin_amdgcn_ldexpf(y, -sx);
        }
        const int jc = p ? ra : cb;
        ta = masked(y, p ? pm_ra : pm_cb, u);  // transitions only
        xa = y;
        ha[u * 8 + jc] = y;
      }
      {
        constexpr int u = SEG - 1 - k, p = u & 1;
        float y = yb;
        if constexpr (u % 8 == 4) {
          const int sx = fbs_exp8<p == 0>(xb);
          y = __builtin_amdgcn_ldexpf(y, -sx);
        }
        const int ic = p ? cb : ra;
        check2(ta, masked(y, p ? pm_cb : pm_ra, u));
        xb = y;
        if constexpr (u >= 1) hb[(u - 1) * 8 + ic] = y;
      }
    });
    const int anybad =
        __builtin_amdgcn_ballot_w64((int)(lob < fbs_bits(0x1p-96f)) | (int)(hib > fbs_bits(0x1p96f))) != 0;
    stamp(6);
    // gamma of the segment's steps: lane u = step ts + u with its whole state row (two float4s of each
    // history), one pass and no cross-lane reduction (was 8 passes of lane = (step, state) with an 8-lane sum)
    {
      const int u = lane, t = ts + u;
      if (t < T) {
        const float4 a0 = *reinterpret_cast<const float4*>(ha + u * 8), a1 = *reinterpret_cast<const float4*>(ha + u * 8 + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(hb + u * 8), h1 = *reinterpret_cast<const float4*>(hb + u * 8 + 4);
        float gv[8] = {a0.x * h0.x, a0.y * h0.y, a0.z * h0.z, a0.w * h0.w, a1.x * h1.x, a1.y * h1.y, a1.z * h1.z, a1.w * h1.w};
        float su = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) su += j < Kv ? gv[j] : 0.f;
        const float rs = __builtin_amdgcn_rcpf(su);
        const bool live = t < L;
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = live ? gv[j] * rs : 0.f;
        float* gr = gq + (int64_t)t * K;
        if (K == 8) {
          *reinterpret_cast<float4*>(gr) = make_float4(gv[0], gv[1], gv[2], gv[3]);
          *reinterpret_cast<float4*>(gr + 4) = make_float4(gv[4], gv[5], gv[6], gv[7]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < K) gr[j] = gv[j];
        }
      }
    }
    if (lane == 0) g_flag[w] = anybad;
    stamp(7);
    __syncthreads();
    for (int s = 0; s < nw; ++s) flagged |= g_flag[s];
    if (!flagged) return;
  }

  // ---------------------------------------------------------------- exact path (rare): natural log,
  // max-shifted LSE, both directions renormalised every step (offsets in fp64), the workspace holding
  // alpha [B][T][K] and beta [B][T][K]; then gamma over the whole sequence.  Overwrites phase 3's gamma.
  float* wal = ws + b * (int64_t)T * K;
  float* wbe = ws + B * (int64_t)T * K + b * (int64_t)T * K;
  if (w == 0) {
    double S = 0.0;
    // emissions enter framed by their step's max (e - E_t; E_t into the fp64 offset): e of about -1e3
    // nats would otherwise cost the recursion's values their low bits
    float a;
    {
      const float e0 = cb < K ? Eb[cb] : NEG_INF;
      const float E0 = allred<8, true>(e0, OpMax{});
      a = (cb < K && e0 != NEG_INF) ? log_pi[cb] + (e0 - E0) : NEG_INF;  // state on the inner axis (step 1 odd)
      S += (double)E0;
    }
    {
      const float mx = allred<8, true>(a, OpMax{});
      if (mx == NEG_INF) S = -__builtin_inf();
      else {
        a -= mx;
        S += mx;
      }
      if (ra == 0 && cb < K) wal[cb] = a;
    }
    for (int t = 1; t < L; ++t) {
      const int p = t & 1;
      const int i = p ? cb : ra, j = p ? ra : cb;
      const float A = (i < K && j < K) ? Ab[(int64_t)t * K * K + i * K + j] : NEG_INF;
      const float e = j < K ? Eb[(int64_t)t * K + j] : NEG_INF;
      const float Et = p ? allred<8, false>(e, OpMax{}) : allred<8, true>(e, OpMax{});  // over the j axis
      S += (double)Et;
      const float v = a + A;
      const float mx = p ? allred<8, true>(v, OpMax{}) : allred<8, false>(v, OpMax{});
      const float ex = mx == NEG_INF ? 0.f : expf(v - mx);
      const float su = p ? allred<8, true>(ex, OpAdd{}) : allred<8, false>(ex, OpAdd{});
      float na = (mx == NEG_INF || e == NEG_INF) ? NEG_INF : (mx + logf(su)) + (e - Et);
      const float nm = p ? allred<8, false>(na, OpMax{}) : allred<8, true>(na, OpMax{});
      if (nm == NEG_INF) S = -__builtin_inf();
      else {
        na -= nm;
        S += nm;
      }
      a = na;
      if ((p ? cb : ra) == 0 && j < K) wal[(int64_t)t * K + j] = a;
    }
    // alpha_{L-1}'s state axis: inner for even L-1 (incl. L = 1), outer for odd
    const bool inner = ((L - 1) & 1) == 0;
    const int st = inner ? cb : ra;
    const float x0 = st < K ? a : NEG_INF;
    const float mx = inner ? allred<8, true>(x0, OpMax{}) : allred<8, false>(x0, OpMax{});
    const float ex = mx == NEG_INF ? 0.f : expf(x0 - mx);
    const float su = inner ? allred<8, true>(ex, OpAdd{}) : allred<8, false>(ex, OpAdd{});
    if (lane == 0) logZ[b] = mx == NEG_INF ? NEG_INF : (float)(S + (double)mx + (double)logf(su));
  }
  if (w == (nw > 1 ? 1 : 0)) {
    // beta_{L-1} = 0 on the j axis of step L-1's parity
    const int p0 = (L - 1) & 1;
    float be = ((p0 ? ra : cb) < K) ? 0.f : NEG_INF;
    if ((p0 ? cb : ra) == 0 && (p0 ? ra : cb) < K) wbe[(int64_t)(L - 1) * K + (p0 ? ra : cb)] = 0.f;
    for (int t = L - 1; t >= 1; --t) {
      const int p = t & 1;
      const int i = p ? cb : ra, j = p ? ra : cb;
      const float A = (i < K && j < K) ? Ab[(int64_t)t * K * K + i * K + j] : NEG_INF;
      const float e = j < K ? Eb[(int64_t)t * K + j] : NEG_INF;
      const float Et = p ? allred<8, false>(e, OpMax{}) : allred<8, true>(e, OpMax{});  // over the j axis
      const float v = (A + (e == NEG_INF ? NEG_INF : e - Et)) + be;
      const float mx = p ? allred<8, false>(v, OpMax{}) : allred<8, true>(v, OpMax{});
      const float ex = mx == NEG_INF ? 0.f : expf(v - mx);
      const float su = p ? allred<8, false>(ex, OpAdd{}) : allred<8, true>(ex, OpAdd{});
      float nb = mx == NEG_INF ? NEG_INF : mx + logf(su);
      const float nm = p ? allred<8, true>(nb, OpMax{}) : allred<8, false>(nb, OpMax{});
      if (nm != NEG_INF) nb -= nm;
      be = nb;
      if ((p ? ra : cb) == 0 && i < K) wbe[(int64_t)(t - 1) * K + i] = be;
    }
  }
  __syncthreads();
  for (int t = (int)threadIdx.x; t < T; t += (int)blockDim.x) {
    float* gt = gq + (int64_t)t * K;
    if (t >= L) {
      for (int j = 0; j < K; ++j) gt[j] = 0.f;
      continue;
    }
    float xs[8];
    float mx = NEG_INF;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xs[j] = j < K ? wal[(int64_t)t * K + j] + wbe[(int64_t)t * K + j] : NEG_INF;
      mx = fmaxf(mx, xs[j]);
    }
    float su = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xs[j] = (mx == NEG_INF || j >= K) ? 0.f : expf(xs[j] - mx);
      su += xs[j];
    }
    for (int j = 0; j < 8; ++j)
      if (j < K) gt[j] = mx == NEG_INF ? __builtin_nanf("") : xs[j] / su;
  }
}

// VQHMM_FB_SEG=0: never the segmented kernel (a test switch read per call, like VQHMM_FB_RES)
bool fwdbwd_seg_ok(int64_t B, int64_t T, int64_t K) {
  const char* env = VQHMM_ENV("VQHMM_FB_SEG");
  if (env && env[0] == '0') return false;
  const bool force = env && env[0] == '1';  // tests: every K <= 8, every T <= 1024
  if (B < 1 || K < 1 || K > 8 || T > (int64_t)FBS_SEG * FBS_MAXW || B > 0x7fffffff) return false;
  // measured against hmm.hip's kernels (tools/kbench.py, profiles/r06/fwdbwd/kbench_smallk.txt): faster at every
  // K >= 2 for T >= 128 except K = 4 at T <= 256, where hmm.hip's 4-lane groups win (B = 1024, T = 200: 25.6 vs
  // 28.2 us)
  return force || (K >= 2 && T >= 2 * FBS_SEG && (K != 4 || T > 4 * FBS_SEG));
}

int launch_fwdbwd_seg(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                      int64_t T, int64_t K, float* gamma, float* logZ, float* ws, hipStream_t s) {
  const int nw = (int)cdiv(T, FBS_SEG);
  static const bool prof = [] {  // profiling build: phase stamps into the workspace (tools/fbseg_prof.py)
    const char* e = VQHMM_PROF_ENV("VQHMM_FB_PROF");
    return e && e[0] == '1';
  }();
  fwdbwd_seg_kernel<<<dim3((unsigned)B), dim3(64 * nw), fbs_lds_bytes(nw), s>>>(
      log_pi, log_A, em, lengths, B, (int)T, (int)K, gamma, logZ, ws, prof ? (unsigned long long*)ws : nullptr);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
