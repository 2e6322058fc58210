// HMM recursions over the Prior's tables.
//
// Semantic sources (no reference code): math.md:23-67 (pi, row-stochastic A_t
// conditioned on u_t), Prior.forward VQ_VAE_HMM_fixed.py:59-71 (log_pi,
// log_A (B,T,K,K)), transition indexing log_A[:, t] = t-1 -> t (:125-127).
// Exact contracts: include/vqhmm.h and oracle/hmm_ref.py.
//
// Lane mapping (K <= 8, KP = next pow2 >= K): a group of G = KP*KP lanes owns
// one sequence (SPW = 64 / G sequences per wave) and holds a step's whole K x K
// transition block, one (i, j) entry per lane.  The (i, j) <-> lane map
// ALTERNATES between steps ("outer" on even t: i = g / KP, j = g % KP; "inner"
// on odd t: i = g % KP, j = g / KP): after reducing over i, the value for state
// j sits in every lane whose j-coordinate is j, which is exactly where the next
// step needs it as its i-coordinate — no broadcast.  The reductions are DPP
// (quad_perm / row_half_mirror / row_ror) and gfx950 permlane16/32 swaps: no
// LDS round trip on the serial chain.
//
// The recursion is serial in t, so a step must never wait for memory: the
// tables stream through a per-wave LDS ring of R chunks of HC steps, filled by
// LDS-DMA loads (global_load_lds, 16 B per lane when K % 4 == 0) issued R - 1
// chunks ahead and retired with a counted `s_waitcnt vmcnt` (the loads never
// drain inside the loop).  Every step then reads its A entry and emission from
// LDS, off the dependency chain.
//
// Viterbi stores, per step, the 64-bit ballot of the lanes that attain the
// max (one SGPR pair → two writelanes into a 64-step register buffer, one
// 512-B store per 64 steps).  The backtrace runs on all 64 lanes: each lane
// composes the backpointer maps of its slice of steps into one byte-permutation
// (v_perm_b32), a 64-step serial resolve links the slices, then every lane
// writes its slice of the path.
// Sequences are independent: no inter-workgroup communication.
#include "hmm_lanes.h"
#include "prof.h"

namespace vqhmm {


template <int K, bool W16>
__global__ __launch_bounds__(64) void viterbi_kernel(const float* __restrict__ log_pi, const float* __restrict__ log_A,
                                                     const float* __restrict__ em,
                                                     const int64_t* __restrict__ lengths, int64_t B, int T,
                                                     int32_t* __restrict__ path, float* __restrict__ score,
                                                     uint2* __restrict__ masks) {
  using Gm = Geo<K, W16>;
  using Rg = Ring<K, W16>;
  constexpr int KP = Gm::KP, G = Gm::G, SPW = Gm::SPW, R = Rg::R, HC = Gm::HC;
  __shared__ float ring[R * Gm::SLOT];  // the only LDS object (keeps hipcc's LDS-DMA waits counted)

  const int lane = threadIdx.x, grp = lane / G, g = lane % G;
  const int64_t b0 = (int64_t)blockIdx.x * SPW;
  const int64_t b = b0 + grp;
  const bool live = b < B;
  const int64_t Lr = live ? lengths[b] : 0;
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  const int i0 = g % KP;
  const float lp = i0 < K ? log_pi[i0] : 0.f;
  int Lmax = L;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) Lmax = max(Lmax, __shfl_xor(Lmax, o));
  Lmax = __builtin_amdgcn_readfirstlane(Lmax);
  wait_vm<0>();  // ordinary loads retired before the LDS-DMA stream starts
  const int Tr = (int)cdiv(T, 64) * 64;
  uint2* wmask = masks + (size_t)blockIdx.x * Tr;

  const LaneMap<K, W16> lm(grp, g);
  const int nchunks = (int)cdiv(Lmax, HC);
  float d = NEG_INF;
  if (nchunks > 0) {
#pragma unroll
    for (int c = 0; c < R - 1; ++c)
      stage_chunk<K, W16>(log_A, em, b0, B, T, min(c, nchunks - 1), ring + c * Gm::SLOT, lane);
  }
  int Lmin = L;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) Lmin = min(Lmin, __shfl_xor(Lmin, o));
  Lmin = __builtin_amdgcn_readfirstlane(Lmin);
  uint32_t mlo = 0, mhi = 0;
  // A / em values of a chunk are read from LDS up front (one wait per chunk),
  // then the max-plus chain runs on registers only.  (Reading the next chunk
  // during this one was measured worse: lgkmcnt counts only 15, and hipcc
  // shuffles the ping-pong sets through copies that wait early.)  Ballots are
  // kept in SGPRs for 8 steps and moved into the mask VGPRs in one batch (one
  // hazard pad per 8 steps instead of one per step).
  constexpr int HB = 8;  // ballots per hazard-padded writelane batch
  auto read_vals = [&](const float* sl, float* av, float* ev) {
#pragma unroll
    for (int s = 0; s < HC; ++s) {
      const int p = s & 1;  // parity of t (t0 even)
      av[s] = lm.a_ok[p] ? sl[lm.a_off[p] + s * K * K] : NEG_INF;
      ev[s] = lm.e_ok[p] ? sl[lm.e_off[p] + s * K] : 0.f;
    }
  };
  // CHECK: some sequence of the wave ends inside this chunk
  auto run_chunk = [&](const float* av, const float* ev, int t0, bool first, auto check) {
    constexpr bool CHECK = decltype(check)::value;
    static_for<HC / 8>([&](auto hi) {
      constexpr int h = decltype(hi)::value;
      uint64_t bal[HB];
      static_for<HB>([&](auto si) {
        constexpr int s = h * HB + decltype(si)::value, p = s & 1;
        if (s == 0 && first) {
          // delta_0 on the inner axis: lane's i0 = g % KP = the even map's j
          d = (L > 0 && i0 < K) ? lp + ev[0] : NEG_INF;
          bal[0] = 0;
          return;
        }
        const float v = d + av[s];
        const float m = p == 0 ? allred<KP, false>(v, OpMax{}) : allred<KP, true>(v, OpMax{});
        bal[s - h * HB] = __builtin_amdgcn_ballot_w64(v == m);
        if (!CHECK || t0 + s < L) d = m + ev[s];
      });
      writelane8<h * HB>(mlo, mhi, bal);
    });
  };
  auto do_chunk = [&](int c, const float* av, const float* ev) {
    const int t0 = c * HC;
    if (t0 + HC <= Lmin) run_chunk(av, ev, t0, c == 0, std::false_type{});
    else run_chunk(av, ev, t0, c == 0, std::true_type{});
    if (lane < HC) wmask[t0 + lane] = make_uint2(mlo, mhi);  // masks of steps t0 .. t0 + HC - 1
  };
  float av[HC], ev[HC];
  for (int c = 0; c < nchunks; ++c) {
    stage_chunk<K, W16>(log_A, em, b0, B, T, min(c + R - 1, nchunks - 1), ring + ((c + R - 1) % R) * Gm::SLOT,
                        lane);
    wait_vm<Rg::WAIT>();
    read_vals(ring + (c % R) * Gm::SLOT, av, ev);
    do_chunk(c, av, ev);
  }

  // final state: first arg-max over the state axis the lanes hold after step L-1
  const int tl = L - 1;
  const bool held_inner = (tl <= 0) || ((tl & 1) == 0);
  const int st = held_inner ? g % KP : g / KP;
  float best = (st < K) ? d : NEG_INF;
  int arg = st;
  if (held_inner) allargmax<KP, true>(best, arg); else allargmax<KP, false>(best, arg);

  // ---- backtrace, one sequence at a time on all 64 lanes, in windows of WT steps
  // staged from the mask stream into the (now idle) ring
  __builtin_amdgcn_s_waitcnt(0);
  __threadfence_block();
  constexpr int WT = (R * Gm::SLOT * 4 / 8) / 64 * 64;
  static_assert(WT >= 64, "ring too small for a mask window");
  uint2* wl = reinterpret_cast<uint2*>(ring);
  for (int q = 0; q < SPW; ++q) {
    const int64_t bq = b0 + q;
    if (bq >= B) break;
    const int Lq = __builtin_amdgcn_readlane(L, q * G);
    const int sq = __builtin_amdgcn_readlane(arg, q * G);
    const float scq = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, best), q * G));
    int32_t* P = path + bq * (int64_t)T;
    for (int t = max(Lq, 0) + lane; t < T; t += 64) P[t] = -1;
    if (lane == 0) score[bq] = Lq > 0 ? scq : NEG_INF;
    if (Lq <= 0) continue;
    if (lane == 0 && Lq == 1) P[0] = sq;
    int state = sq;  // state at the top step of the current window (wave-uniform)
    // mask steps 1 .. Lq-1; windows [w0, w0 + WT) from the top down
    for (int w0 = ((Lq - 1) / WT) * WT; Lq > 1 && w0 >= 0; w0 -= WT) {
      const int lo = max(w0, 1), hi = min(w0 + WT - 1, Lq - 1);
      // stage masks [w0, w0 + WT) (whole 64-step blocks)
      __syncthreads();
      const int nblk = (hi - w0) / 64 + 1;
      for (int k = 0; k < 2 * nblk; ++k)  // 64 dwords per instruction
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(wmask + w0) + k * 64 + lane,
                                         (__attribute__((address_space(3))) void*)(reinterpret_cast<uint32_t*>(wl) +
                                                                                   k * 64),
                                         4, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      const int n = hi - lo + 1;
      const int cl = (int)cdiv(n, 64);
      const int clo = lo + lane * cl, chi = min(clo + cl - 1, hi);
      // compose this lane's slice: F maps the state at step chi to the state at step clo - 1
      uint32_t flo = 0x03020100u, fhi = 0x07060504u;
      for (int t = chi; t >= clo; --t) {
        const uint2 mm = wl[t - w0];
        const uint2 mp = bp_map<K>(mm.x, mm.y, q, t & 1);
        flo = perm_bytes(mp, flo);
        fhi = perm_bytes(mp, fhi);
      }
      // serial resolve from the top slice down: end state of each slice
      int ecur = state, mine = 0;
      for (int cc = 63; cc >= 0; --cc) {
        const int slo = lo + cc * cl;
        if (slo > hi) continue;
        mine = lane == cc ? ecur : mine;
        const uint32_t xl = __builtin_amdgcn_readlane((int)flo, cc), xh = __builtin_amdgcn_readlane((int)fhi, cc);
        ecur = (int)((ecur < 4 ? (xl >> (8 * ecur)) : (xh >> (8 * (ecur - 4)))) & 0xFFu);
      }
      // walk: P[t] for t in [clo, chi]; the lowest slice also writes P[lo - 1]
      int s = mine;
      for (int t = chi; t >= clo; --t) {
        P[t] = s;
        const uint2 mm = wl[t - w0];
        const uint2 mp = bp_map<K>(mm.x, mm.y, q, t & 1);
        s = (int)((s < 4 ? (mp.x >> (8 * s)) : (mp.y >> (8 * (s - 4)))) & 0xFFu);
      }
      if (clo == lo && clo <= chi) P[lo - 1] = s;
      state = ecur;
    }
  }
}

size_t viterbi_ws_bytes(int64_t B, int64_t T, int64_t K) {
  if (K > 8 && K <= 32) return viterbi_wide_ws_bytes(B, T);
  if (K > 32) return hmm_generic_supported(K) ? hmm_generic_viterbi_ws_bytes(B, T, K) : 0;
  if (K < 1 || K > 8) return 0;
  const int KP = K <= 2 ? 2 : K <= 4 ? 4 : 8;
  const int64_t spw = 64 / (KP * KP);
  return (size_t)cdiv(B, spw) * (size_t)cdiv(T, 64) * 64 * 8;
}

template <int K, bool W16>
static void viterbi_go(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                       int64_t T, int32_t* path, float* score, void* ws, hipStream_t s) {
  const dim3 grid((unsigned)cdiv(B, Geo<K, W16>::SPW));
  viterbi_kernel<K, W16><<<grid, 64, 0, s>>>(log_pi, log_A, em, lengths, B, (int)T, path, score, (uint2*)ws);
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int launch_viterbi(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                   int64_t T, int64_t K, int32_t* path, float* score, void* ws, size_t ws_bytes, hipStream_t s) {
  if (B == 0) return VQHMM_OK;
  if (K < 1 || !hmm_generic_supported(K) || T < 1 || T > (1 << 28)) return VQHMM_EUNSUPPORTED;
  if (!ws || ws_bytes < viterbi_ws_bytes(B, T, K)) return VQHMM_EWORKSPACE;
  if (K > 32) return launch_viterbi_generic(log_pi, log_A, em, lengths, B, T, K, path, score, ws, s);
  if (K > 8) return launch_viterbi_wide(log_pi, log_A, em, lengths, B, T, K, path, score, ws, s);
  const bool w16 = aligned16(log_A) && aligned16(em);
  switch (K) {
    case 1: viterbi_go<1, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s); break;
    case 2: viterbi_go<2, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s); break;
    case 3: viterbi_go<3, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s); break;
    case 4:
      if (w16) viterbi_go<4, true>(log_pi, log_A, em, lengths, B, T, path, score, ws, s);
      else viterbi_go<4, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s);
      break;
    case 5: viterbi_go<5, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s); break;
    case 6: viterbi_go<6, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s); break;
    case 7: viterbi_go<7, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s); break;
    default:
      if (w16) viterbi_go<8, true>(log_pi, log_A, em, lengths, B, T, path, score, ws, s);
      else viterbi_go<8, false>(log_pi, log_A, em, lengths, B, T, path, score, ws, s);
      break;
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}


// ------------------------------------------------------------ forward-backward
// One workgroup = 2 waves on the same SPW sequences: wave 0 runs alpha (t
// ascending) and wave 1 beta (t descending) at the same time, each streaming
// the tables through its own ring; both stage their per-step vectors in LDS and
// flush one chunk at a time to the workspace; then both waves form gamma in
// parallel over t (no serial dependency left).
//
// Everything runs in base 2 (lg = log2; inputs scaled by log2(e) as they are
// read) with shifts — arbitrary constants of a shift-invariant recursion,
// chosen so every vector stays within a few steps' spread of 0:
//   alpha: al_0 = lg pi + (lg e_0 - E_0),
//          al_t(j) = lg sum_i 2^(al_{t-1}(i) + lg A_t(i,j)) + (lg e_t(j) - E_t) - mu_t
//          with E_t = max_j lg e_t(j) (from the staged tables, off the chain) and
//          mu_t = max_i al_{t-1}(i) every FB_NORM-th step (reduced beside the chain), else 0;
//          logZ = ln2 (sum_t mu_t + lg sum_j 2^al_{L-1}(j)) + sum_t max_j e_t(j)
//   beta:  be_{L-1} = 0,
//          be_t(i) = lg sum_j 2^((lg A_{t+1}(i,j) + lg e_{t+1}(j) - E_{t+1}) + be_{t+1}(j)) - nu_t,
//          nu_t = max_j be_{t+1}(j) every FB_NORM-th step, else 0
//   gamma_t(i) = softmax_i(al_t(i) + be_t(i))
// With the shifts, a step's terms stay within a few steps' transition and
// emission spread of 1, so the serial chain skips the max-subtraction of a
// log-sum-exp: add, exp2, the add-reduction, log2, add.  A chunk in which a
// live step's column sum leaves [2^-FB_LIM, 2^FB_LIM] (an over/underflow that
// may have dropped a significant term, or an all -inf column) is recomputed
// from its saved start state with the max-shifted log-sum-exp, normalised
// every step — same contract, rare path.
//
// Linear tier (tried first on every chunk).  Inside a chunk the recursions run on
// x = 2^(al - frame) with the per-step table m(i, j) = 2^((lg A(i,j) + lg e(j)) lg e)
// precomputed off the chain, so a step is one multiply and the add-reduction:
//   alpha: x_t(j) = sum_i x_{t-1}(i) m_t(i, j),   beta: x_t(i) = sum_j m_{t+1}(i, j) x_{t+1}(j)
// Every FB_LNORM-th step rescales by 2^-k, k = the exponent of the running max (exact, a
// power of two; its max-reduction runs beside the chain's add-reduction).  The chunk starts
// from the log-domain state (x = 2^(al - max al)) and ends by converting back (al = lg x), so
// chunk boundaries keep the log-domain range.  A chunk in which some live entry leaves
// [2^-FB_LIM, 2^FB_LIM] (nothing below 2^-126 can then have carried weight) falls back to the
// log tier above from the saved start state.  The per-step stores are lg x: a per-step
// constant offset, which gamma's softmax over the states cancels.
// Workspace: al [B][T][K], then be' [B][T][K] with be'[t+1] = be_t (base 2).
constexpr float F32_LOWEST = -3.402823466e38f;
constexpr float LOG2E_F = 1.44269504088896341f;
constexpr double LN2_D = 0.69314718055994531;
constexpr float FB_LIM = 96.f;  // fast-step column sums must stay within 2^(+-FB_LIM)
constexpr int FB_NORM = 4;      // fast steps renormalise by the running max every FB_NORM steps
constexpr int FB_LNORM = 8;     // the linear tier rescales every FB_LNORM steps (and at each chunk start)

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float flog2(float x) { return __builtin_amdgcn_logf(x); }

// the linear tier's per-step table of a staged chunk (alpha: step s has the parity of t = s;
// beta: data step s serves t = s - 1)
template <int K, bool W16, bool BETA>
__device__ __forceinline__ void read_lin_chunk(const float* sl, const LaneMap<K, W16>& lm, float* ml) {
  using Gm = Geo<K, W16>;
  constexpr int HC = Gm::HC;
#pragma unroll
  for (int s = 0; s < HC; ++s) {
    const int p = (s + (BETA ? 1 : 0)) & 1;
    const float a = lm.a_ok[p] ? sl[lm.a_off[p] + s * K * K] : NEG_INF;
    const float e = lm.e_ok[p] ? sl[lm.e_off[p] + s * K] : 0.f;
    ml[s] = fexp2((a + e) * LOG2E_F);
  }
}

// out-of-range test of the linear tier's live entries
__device__ __forceinline__ bool lin_bad(float lo, float hi) { return !(lo >= 0x1p-96f) || !(hi <= 0x1p96f); }

template <int N>
__device__ __forceinline__ float tree_sum(const float* v) {  // pairwise (fixed order)
  float t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = v[i];
#pragma unroll
  for (int w = N / 2; w >= 1; w /= 2)
#pragma unroll
    for (int i = 0; i < w; ++i) t[i] += t[i + w];
  return t[0];
}

// a staged chunk into registers (base 2), read up front off the chain.  Per step:
//   alpha: av = lg A(i,j), dv = lg e(j) - E, xv = max_j e (natural log)
//   beta:  av = lg A(i,j) + lg e(j) - E      (data step d serves t = d - 1)
template <int K, bool W16, bool BETA>
__device__ __forceinline__ void read_fb_chunk(const float* sl, const LaneMap<K, W16>& lm, float* av, float* dv,
                                              float* xv) {
  using Gm = Geo<K, W16>;
  constexpr int KP = Gm::KP, HC = Gm::HC;
#pragma unroll
  for (int s = 0; s < HC; ++s) {
    const int p = (s + (BETA ? 1 : 0)) & 1;  // parity of the step's t
    const float a = lm.a_ok[p] ? sl[lm.a_off[p] + s * K * K] : NEG_INF;
    const float e = lm.e_ok[p] ? sl[lm.e_off[p] + s * K] : 0.f;
    // the outer map's j = g % KP covers every state along the inner axis
    const float ein = lm.e_ok[0] ? sl[lm.e_off[0] + s * K] : NEG_INF;
    float emx = allred<KP, true>(ein, OpMax{});
    emx = emx == NEG_INF ? 0.f : emx;
    if constexpr (BETA) {
      av[s] = (a + (e - emx)) * LOG2E_F;
    } else {
      av[s] = a * LOG2E_F;
      dv[s] = (e - emx) * LOG2E_F;
      xv[s] = emx;
    }
  }
}

// FUSE (round 4): gamma formed beside the chains, as the resident kernel forms it.  Four waves: the two
// chains and two flush waves; one LDS barrier per chunk iteration pairs alpha's chunk c with beta's data
// chunk nch-1-c, and while the chains run iteration c + 1 the flush waves take iteration c's vectors
// (double-buffered) and form gamma_t where the other direction's value is already in an LDS history (from
// an earlier iteration), keeping their own value there otherwise; the t whose two chunks ran in the same
// iteration follow after the loop.  No workspace and no gamma pass: HBM sees the tables twice and gamma
// once.  The histories take the ring one chunk shallower (fb_fused_ok: two workgroups per CU still fit).
// NSQ = 2 (the default where it fits): ONE 8-wave workgroup per CU pair of sequence groups, waves 0-3 the
// four chains (alpha / beta of group 0, then of group 1) so that each chain has a SIMD of its own, at
// raised priority, and waves 4-7 their flush waves beside them.  Two 4-wave workgroups per CU instead put
// their waves on the same SIMDs, two chains sharing one (measured below).  Both groups run the
// workgroup's longest chunk count, so the barrier counts agree; a group past its own length keeps its
// state, as lanes of one wave with different lengths already do.
template <int K, bool W16>
struct FbStream {
  using Gm = Geo<K, W16>;
  using Rg = Ring<K, W16>;
  static constexpr bool CAN_FUSE = Rg::R >= 3;
  static constexpr int VB = Gm::SPW * Gm::HC * Gm::KP;
  __host__ __device__ static constexpr int ring(bool fuse) { return fuse ? Rg::R - 1 : Rg::R; }
  __host__ __device__ static constexpr int pw(bool fuse) { return ring(fuse) * Gm::SLOT + (fuse ? 2 : 1) * VB; }
  __host__ __device__ static int hh(int T) { return ((T + Gm::HC - 1) / Gm::HC / 2 + 1) * Gm::HC; }
  // LDS floats of one sequence group (a multiple of 4: every group's base stays 16-B aligned)
  __host__ __device__ static int group_floats(bool fuse, int T) {
    return 2 * pw(fuse) + (fuse ? 2 * Gm::SPW * hh(T) * Gm::KP + 4 : 0);
  }
  static size_t lds_bytes(bool fuse, int T) { return (size_t)group_floats(fuse, T) * sizeof(float); }
};

template <int K, bool W16, bool FUSE, int NSQ = 1>
__global__ __launch_bounds__(FUSE ? 256 * NSQ : 128) void fwdbwd_kernel(const float* __restrict__ log_pi,
                                                     const float* __restrict__ log_A, const float* __restrict__ em,
                                                     const int64_t* __restrict__ lengths, int64_t B, int T,
                                                     float* __restrict__ gamma, float* __restrict__ logZ,
                                                     float* __restrict__ ws, int lin_tier, int no_gamma) {
  using Gm = Geo<K, W16>;
  using Rg = Ring<K, W16>;
  using FS = FbStream<K, W16>;
  static_assert(!FUSE || FS::CAN_FUSE, "fused gamma needs a ring of three chunks or more");
  static_assert(NSQ == 1 || (FUSE && NSQ == 2), "two sequence groups per workgroup: fused form only");
  constexpr int KP = Gm::KP, G = Gm::G, SPW = Gm::SPW, R = FS::ring(FUSE), HC = Gm::HC;
  constexpr int RWAIT = Rg::NI * (R - 1);  // the ring's counted wait: R - 1 chunks stay in flight
  constexpr int VB = FS::VB;              // per-wave vector buffer [SPW][HC][KP] (floats)
  constexpr int PW = FS::pw(FUSE);        // LDS floats per wave
  extern __shared__ float4 smem_fbs[];
  const int hwave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // NSQ = 2: sequence group sq, role wave (0 alpha, 1 beta, 2 / 3 their flush waves)
  const int sq = NSQ == 1 ? 0 : (hwave < 4 ? hwave >> 1 : (hwave - 4) >> 1);
  const int wave = NSQ == 1 ? hwave : (hwave < 4 ? (hwave & 1) : 2 + (hwave & 1));
  // one sequence group's LDS: [2][PW] (+ FUSE: the two histories and the flags)
  float* lds = reinterpret_cast<float*>(smem_fbs) + (NSQ == 1 ? 0 : sq * FS::group_floats(FUSE, T));
  if (NSQ == 2 && wave < 2) __builtin_amdgcn_s_setprio(2);  // the chains first on the SIMD they share

  const int lane = threadIdx.x & 63, grp = lane / G, g = lane % G;
  const int64_t b0 = ((int64_t)blockIdx.x * NSQ + sq) * SPW;
  const int64_t b = b0 + grp;
  const bool live = b < B;
  const int64_t Lr = live ? lengths[b] : 0;
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  const int jo = g % KP, ji = g / KP;  // lane's inner / outer coordinate
  const float lp2 = jo < K ? log_pi[jo] * LOG2E_F : 0.f;
  int Lmax = L, Lmin = L;
  if constexpr (NSQ == 2) {  // the workgroup's chunk count: over the other group's lengths too
    const int64_t bo = ((int64_t)blockIdx.x * NSQ + (sq ^ 1)) * SPW + grp;
    const int64_t Lo = bo < B ? lengths[bo] : 0;
    const int Lc = (int)(Lo <= 0 ? 0 : (Lo < T ? Lo : T));
    Lmax = max(Lmax, Lc);  // (Lmin stays the group's own: it only picks the unchecked step form)
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    Lmax = max(Lmax, __shfl_xor(Lmax, o));
    Lmin = min(Lmin, __shfl_xor(Lmin, o));
  }
  Lmax = __builtin_amdgcn_readfirstlane(Lmax);
  Lmin = __builtin_amdgcn_readfirstlane(Lmin);
  wait_vm<0>();
  float* ring = lds + (wave & 1) * PW;
  float* vbuf = ring + R * Gm::SLOT;  // (FUSE: two buffers, chunk c in vbuf + (c & 1) VB)
  float* vrow = vbuf + grp * HC * KP;
  float* ws_al = ws;
  float* ws_be = ws + (size_t)B * T * K;
  const LaneMap<K, W16> lm(grp, g);
  const int nchunks = (int)cdiv(Lmax, HC);

  // flush vbuf -> dst rows [t0, t0 + HC) of the wave's sequences (t < T only).
  // Every lane of a group stores its step value unmasked (lanes sharing a
  // state write the same word); the wave's LDS ops retire in order.
  auto flush = [&](float* dst, int t0, bool linear) {
    asm volatile("" ::: "memory");
    constexpr int NF = (VB + 63) / 64;
#pragma unroll
    for (int k = 0; k < NF; ++k) {
      const int idx = k * 64 + lane;
      if (VB % 64 == 0 || idx < VB) {
        const int q = idx / (HC * KP), r = idx - q * (HC * KP), s = r / KP, j = r - s * KP;
        const float v = linear ? flog2(vbuf[idx]) : vbuf[idx];
        if (j < K && b0 + q < B && t0 + s < T) dst[((b0 + q) * (int64_t)T + t0 + s) * K + j] = v;
      }
    }
    asm volatile("" ::: "memory");
  };
  // ---- FUSE: the two histories and the flushes that form gamma (fwdbwd_resident_kernel's rules)
  const int nchT = (int)cdiv(T, HC), HH = FS::hh(T);
  (void)nchT;
  float* hist_a = lds + 2 * PW;                 // al_t at [q][t][state], t < HH
  float* hist_b = hist_a + SPW * HH * KP;        // be'[d] at [q][d - dbase][state]
  const int dbase = ((nchunks - 1) / 2) * HC;    // first data step kept in hist_b
  constexpr int NF = VB / 64;
  static_assert(!FUSE || VB % 64 == 0, "flush covers whole wave passes");
  int* fflags = reinterpret_cast<int*>(hist_b + SPW * HH * KP);  // [chain][buffer]: the chunk ran the linear tier
  auto seqlen = [&](int q) {
    const int64_t bq = b0 + q;
    if (bq >= B) return -1;
    const int64_t l = lengths[bq];
    return (int)(l <= 0 ? 0 : (l < T ? l : T));
  };
  int Lfl[FUSE ? NF : 1];
  if constexpr (FUSE) {
#pragma unroll
    for (int r = 0; r < NF; ++r) Lfl[r] = seqlen((r * 64 + lane) / (HC * KP));
  }
  // softmax over the KP-lane state group of lanes idx % KP (padding states masked)
  auto store_gamma = [&](int q, int t, int j, float xs, bool own) {
    const float xm = (j < K) ? xs : NEG_INF;
    const float mx = allred<KP, true>(xm, OpMax{});
    const float ex = (j < K && mx != NEG_INF) ? fexp2(xm - mx) : 0.f;
    const float sm = allred<KP, true>(ex, OpAdd{});
    if (own && j < K) gamma[((b0 + q) * (int64_t)T + t) * K + j] = ex * __builtin_amdgcn_rcpf(sm);
  };
  auto flush_alpha_f = [&](int c, bool linear, const float* vb) {
#pragma unroll
    for (int r = 0; r < NF; ++r) {
      const int idx = r * 64 + lane;
      const int q = idx / (HC * KP), rr = idx - q * (HC * KP), s = rr / KP, j = rr - s * KP;
      const int t = c * HC + s;
      const float v = linear ? flog2(vb[idx]) : vb[idx];
      if (t < HH) hist_a[(q * HH + t) * KP + j] = v;
      const int Lq = Lfl[r];
      const bool ok = Lq >= 0 && t < T;
      const bool own = ok && (t >= Lq - 1 || t / HC + (t + 1) / HC >= nchunks);
      const bool past = ok && t >= Lq;  // gamma_t = 0 past the sequence
      float xs = v;
      if (own && t < Lq - 1) xs += hist_b[(q * HH + (t + 1 - dbase)) * KP + j];
      store_gamma(q, t, j, xs, own && !past);
      if (past && j < K) gamma[((b0 + q) * (int64_t)T + t) * K + j] = 0.f;
    }
  };
  auto flush_beta_f = [&](int k, bool linear, const float* vb) {
#pragma unroll
    for (int r = 0; r < NF; ++r) {
      const int idx = r * 64 + lane;
      const int q = idx / (HC * KP), rr = idx - q * (HC * KP), s = rr / KP, j = rr - s * KP;
      const int d = k * HC + s, t = d - 1;
      const float v = linear ? flog2(vb[idx]) : vb[idx];
      if (d >= dbase && d - dbase < HH) hist_b[(q * HH + (d - dbase)) * KP + j] = v;
      const int Lq = Lfl[r];
      const bool own = Lq >= 0 && t >= 0 && t < Lq - 1 && t / HC + d / HC <= nchunks - 2;
      const float xs = own ? hist_a[(q * HH + t) * KP + j] + v : 0.f;
      store_gamma(q, t, j, xs, own);
    }
  };

  float av[HC], dv[HC], xv[HC], mv[HC], ml[HC];
  float rng = 0.f;  // max |lg column sum| over the chunk's live fast steps
  float x = 0.f, lo = 1.f, hi = 1.f;  // linear tier: chain value, range of the live entries

  if (wave == 0) {
    // ------------------------------------------------------------ alpha
    if (nchunks > 0) {
#pragma unroll
      for (int c = 0; c < R - 1; ++c)
        stage_chunk<K, W16>(log_A, em, b0, B, T, min(c, nchunks - 1), ring + c * Gm::SLOT, lane);
    }
    float al = NEG_INF;
    double S2 = 0.0, SE = 0.0;  // sum of mu (base 2), sum of E (natural)
    // EXACT: max-shifted log-sum-exp; CHECK: some sequence ends inside the chunk
    auto steps = [&](int t0, bool first, auto exact, auto check) {
      constexpr bool EXACT = decltype(exact)::value, CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = decltype(si)::value, p = s & 1;
        if (s == 0 && first) {  // al_0 on the inner axis: lane's i = g % KP = the even map's j
          al = (L > 0 && jo < K) ? lp2 + dv[0] : NEG_INF;
          mv[0] = 0.f;
          vrow[jo] = al;
          return;
        }
        const bool upd = !CHECK || t0 + s < L;
        const float v = al + av[s];
        float mus = 0.f;
        if constexpr (EXACT || s % FB_NORM == 0) {
          const float mu = allred<KP, p == 1>(al, OpMax{});
          mus = mu == NEG_INF ? 0.f : mu;
        }
        float nal;
        if constexpr (EXACT) {
          const float mm = fmaxf(allred<KP, p == 1>(v, OpMax{}), F32_LOWEST);
          const float sm = allred<KP, p == 1>(fexp2(v - mm), OpAdd{});
          nal = (mm + flog2(sm)) + (dv[s] - mus);
        } else {
          const float ls = flog2(allred<KP, p == 1>(fexp2(v), OpAdd{}));
          nal = ls + (dv[s] - mus);
          rng = fmaxf(rng, fabsf((lm.e_ok[p] && upd) ? ls : 0.f));
        }
        mv[s] = upd ? mus : 0.f;
        if (upd) al = nal;
        vrow[s * KP + (p == 0 ? jo : ji)] = al;  // state j = the lane's j-coordinate
      });
    };
    // linear tier (see above); sk = the chunk's frame shifts (base 2)
    float sk = 0.f;
    auto lin_steps = [&](int t0, bool first, float e0, auto check) {
      constexpr bool CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = decltype(si)::value, p = s & 1;
        if (s == 0 && first) {  // x_0 on the inner axis from al_0 = lg pi + lg e_0
          const float a0 = (L > 0 && jo < K) ? lp2 + e0 : NEG_INF;
          const float m0 = allred<KP, true>(a0, OpMax{});
          const float m0s = m0 == NEG_INF ? 0.f : m0;
          x = fexp2(a0 - m0s);
          sk = m0s;
          if (L > 0 && jo < K) lo = fminf(lo, x);
          vrow[jo] = x;
          return;
        }
        const bool upd = !CHECK || t0 + s < L;
        const float v = x * ml[s];
        int k = 0;
        if constexpr (s % FB_LNORM == FB_LNORM / 2) k = __builtin_amdgcn_frexp_expf(allred<KP, p == 1>(x, OpMax{}));
        float y = allred<KP, p == 1>(v, OpAdd{});
        if constexpr (s % FB_LNORM == FB_LNORM / 2) y = __builtin_amdgcn_ldexpf(y, -k);
        const bool chk = upd && lm.e_ok[p];
        lo = chk ? fminf(lo, y) : lo;
        hi = chk ? fmaxf(hi, y) : hi;
        if (upd) {
          x = y;
          sk += (float)k;
        }
        vrow[s * KP + (p == 0 ? jo : ji)] = x;
      });
    };
    for (int c = 0; c < nchunks; ++c) {
      if constexpr (FUSE) vrow = vbuf + (c & 1) * VB + grp * HC * KP;
      stage_chunk<K, W16>(log_A, em, b0, B, T, min(c + R - 1, nchunks - 1), ring + ((c + R - 1) % R) * Gm::SLOT,
                          lane);
      wait_vm<RWAIT>();
      const float* sl = ring + (c % R) * Gm::SLOT;
      const int t0 = c * HC;
      const float al_c = al;
      bool linear = false;
      if (lin_tier) {
        read_lin_chunk<K, W16, false>(sl, lm, ml);
        const float e0 = c == 0 && lm.e_ok[0] ? sl[lm.e_off[0]] * LOG2E_F : NEG_INF;
        lo = hi = 1.f;
        if (c > 0) {  // state of step t0 - 1 (odd: outer axis) -> its frame
          const float m = allred<KP, false>(al, OpMax{});
          const float ms = m == NEG_INF ? 0.f : m;
          x = fexp2(al - ms);
          sk = ms;
          if (t0 < L && ji < K) lo = fminf(lo, x);
        }
        if (t0 + HC <= Lmin) lin_steps(t0, c == 0, e0, std::false_type{});
        else lin_steps(t0, c == 0, e0, std::true_type{});
        linear = !__builtin_amdgcn_ballot_w64(lin_bad(lo, hi));
      }
      if (linear) {
        if (t0 < L) {  // (a sequence that ended before the chunk keeps its state; its axis is not the outer one)
          al = flog2(x);
          S2 += (double)sk;
        }
      } else {
        read_fb_chunk<K, W16, false>(sl, lm, av, dv, xv);
        al = al_c;
        rng = 0.f;
        if (t0 + HC <= Lmin) steps(t0, c == 0, std::false_type{}, std::false_type{});
        else steps(t0, c == 0, std::false_type{}, std::true_type{});
        if (__builtin_amdgcn_ballot_w64(rng > FB_LIM)) {  // rare: recompute the chunk exactly
          al = al_c;
          steps(t0, c == 0, std::true_type{}, std::true_type{});
        }
#pragma unroll
        for (int s = 0; s < HC; ++s) xv[s] = t0 + s < L ? xv[s] : 0.f;
        S2 += (double)tree_sum<HC>(mv);
        SE += (double)tree_sum<HC>(xv);
      }
      if constexpr (FUSE) {
        if (lane == 0) fflags[c & 1] = linear;
        lds_barrier();  // chunk c to the flush waves (they take it while this wave runs chunk c + 1)
      } else {
        flush(ws_al, t0, linear);
      }
    }
    if constexpr (FUSE) lds_barrier();  // the last chunk flushed
    // logZ from the state axis held after step L-1 (even t: inner)
    const int tl = L - 1;
    const bool held_inner = (tl <= 0) || ((tl & 1) == 0);
    const int st = held_inner ? jo : ji;
    const float x0 = st < K ? al : NEG_INF;
    const float mx = held_inner ? allred<KP, true>(x0, OpMax{}) : allred<KP, false>(x0, OpMax{});
    const float mxs = fmaxf(mx, F32_LOWEST);
    const float ex = fexp2(x0 - mxs);
    const float sx = held_inner ? allred<KP, true>(ex, OpAdd{}) : allred<KP, false>(ex, OpAdd{});
    if (live && g == 0)
      logZ[b] = L > 0 ? (float)(LN2_D * (S2 + (double)mxs + (double)flog2(sx)) + SE)
                      : __builtin_bit_cast(float, 0x7fc00000u);
  } else if (!FUSE || wave == 1) {
    // ------------------------------------------------------------ beta
    // chunk k holds data steps [k HC, k HC + HC); data step d serves beta step t = d - 1
    if (nchunks > 0) {
#pragma unroll
      for (int c = 0; c < R - 1; ++c)
        stage_chunk<K, W16>(log_A, em, b0, B, T, max(nchunks - 1 - c, 0), ring + c * Gm::SLOT, lane);
    }
    float be = 0.f;
    auto steps = [&](int d0, bool last, auto exact, auto check) {
      constexpr bool EXACT = decltype(exact)::value, CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = HC - 1 - decltype(si)::value, p = (s + 1) & 1;  // p = parity of t
        if (s == 0 && last) return;                                       // t = -1
        const bool upd = !CHECK || d0 + s - 1 < L - 1;
        const float v = av[s] + be;
        float nus = 0.f;
        if constexpr (EXACT || s % FB_NORM == 0) {
          const float nu = allred<KP, p == 0>(be, OpMax{});
          nus = nu == NEG_INF ? 0.f : nu;
        }
        float nb;
        if constexpr (EXACT) {
          const float mm = fmaxf(allred<KP, p == 0>(v, OpMax{}), F32_LOWEST);
          const float sm = allred<KP, p == 0>(fexp2(v - mm), OpAdd{});
          nb = (mm + flog2(sm)) - nus;
        } else {
          const float ls = flog2(allred<KP, p == 0>(fexp2(v), OpAdd{}));
          nb = ls - nus;
          rng = fmaxf(rng, fabsf((lm.e_ok[p ^ 1] && upd) ? ls : 0.f));  // e_ok[p^1]: lane's i < K
        }
        if (upd) be = nb;
        vrow[s * KP + (p == 0 ? ji : jo)] = be;  // state i = the lane's i-coordinate; slot s <-> be'[t + 1]
      });
    };
    auto lin_steps = [&](int d0, bool last, auto check) {
      constexpr bool CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = HC - 1 - decltype(si)::value, p = (s + 1) & 1;  // p = parity of t
        if (s == 0 && last) return;                                       // t = -1
        const bool upd = !CHECK || d0 + s - 1 < L - 1;
        const float v = ml[s] * x;
        int kx = 0;
        if constexpr (s % FB_LNORM == FB_LNORM / 2) kx = __builtin_amdgcn_frexp_expf(allred<KP, p == 0>(x, OpMax{}));
        float y = allred<KP, p == 0>(v, OpAdd{});
        if constexpr (s % FB_LNORM == FB_LNORM / 2) y = __builtin_amdgcn_ldexpf(y, -kx);
        const bool chk = upd && lm.e_ok[p ^ 1];
        lo = chk ? fminf(lo, y) : lo;
        hi = chk ? fmaxf(hi, y) : hi;
        if (upd) x = y;
        vrow[s * KP + (p == 0 ? ji : jo)] = x;
      });
    };
    for (int c = 0; c < nchunks; ++c) {
      if constexpr (FUSE) vrow = vbuf + (c & 1) * VB + grp * HC * KP;
      const int k = nchunks - 1 - c;
      stage_chunk<K, W16>(log_A, em, b0, B, T, max(k - (R - 1), 0), ring + ((c + R - 1) % R) * Gm::SLOT, lane);
      wait_vm<RWAIT>();
      const float* sl = ring + (c % R) * Gm::SLOT;
      const int d0 = k * HC;
      const float be_c = be;
      bool linear = false;
      if (lin_tier) {
        read_lin_chunk<K, W16, true>(sl, lm, ml);
        // state of data step d0 + HC (even t = d0 + HC - 1 ... held on the inner axis) -> its frame
        const float m = allred<KP, true>(be, OpMax{});
        x = fexp2(be - (m == NEG_INF ? 0.f : m));
        lo = hi = 1.f;
        if (d0 + HC - 1 < L - 1 && jo < K) lo = fminf(lo, x);
        if (d0 + HC <= Lmin) lin_steps(d0, k == 0, std::false_type{});
        else lin_steps(d0, k == 0, std::true_type{});
        linear = !__builtin_amdgcn_ballot_w64(lin_bad(lo, hi));
      }
      if (linear) {
        be = flog2(x);
      } else {
        read_fb_chunk<K, W16, true>(sl, lm, av, dv, xv);
        be = be_c;
        rng = 0.f;
        if (d0 + HC <= Lmin) steps(d0, k == 0, std::false_type{}, std::false_type{});
        else steps(d0, k == 0, std::false_type{}, std::true_type{});
        if (__builtin_amdgcn_ballot_w64(rng > FB_LIM)) {
          be = be_c;
          steps(d0, k == 0, std::true_type{}, std::true_type{});
        }
      }
      if constexpr (FUSE) {
        if (lane == 0) fflags[2 + (c & 1)] = linear;
        lds_barrier();
      } else {
        flush(ws_be, d0, linear);
      }
    }
    if constexpr (FUSE) lds_barrier();
  } else {
    // ------------------------------------------------------------ (FUSE) flush waves: wave 2 alpha's chunks,
    // wave 3 beta's, one iteration behind the chains
    if constexpr (FUSE) {
      const int ch = wave & 1;
      for (int it = 0; it < nchunks; ++it) {
        lds_barrier();
        const bool lin = fflags[2 * ch + (it & 1)] != 0;
        const float* vb = lds + ch * PW + R * Gm::SLOT + (it & 1) * VB;
        if (ch == 0) flush_alpha_f(it, lin, vb);
        else flush_beta_f(nchunks - 1 - it, lin, vb);
      }
      lds_barrier();
    }
  }

  // ---------------------------------------------------------------- gamma
  // (sequence, t) items spread over both waves, GU per thread with all their loads in flight
  // before the first use
  __syncthreads();
  if constexpr (FUSE) {
    if (wave == 2) {  // the t whose alpha and beta chunks ran in the same iteration: t/HC + (t+1)/HC == nch - 1
      const int tb = max(((nchunks - 1) / 2) * HC - 1, 0);
      for (int idx = lane; idx < SPW * 2 * HC * KP; idx += 64) {  // wave-uniform trip count
        const int q = idx / (2 * HC * KP), rr = idx - q * (2 * HC * KP), s = rr / KP, j = rr - s * KP;
        const int t = tb + s;
        const int Lq = seqlen(q);
        const bool own = Lq >= 0 && t < Lq - 1 && t / HC + (t + 1) / HC == nchunks - 1;
        const float xs =
            own ? hist_a[(q * HH + t) * KP + j] + hist_b[(q * HH + (t + 1 - dbase)) * KP + j] : 0.f;
        store_gamma(q, t, j, xs, own);
      }
    } else if (wave == 3) {  // steps no chain reached: t >= nch * HC
      const int t0 = nchunks * HC, nt = T - t0;
      for (int64_t idx = lane; idx < (int64_t)SPW * nt * K; idx += 64) {
        const int q = (int)(idx / ((int64_t)nt * K));
        const int64_t rr = idx - (int64_t)q * nt * K;
        if (b0 + q < B) gamma[((b0 + q) * (int64_t)T + t0) * K + rr] = 0.f;
      }
    }
    return;
  }
  if (no_gamma) return;  // timing experiment (profiling build, VQHMM_FB_NOGAMMA): gamma left unwritten
  constexpr int GU = 4;
  const int nit = SPW * T;
  for (int base = 0; base < nit; base += 128 * GU) {
    float xs[GU][K];
    int tt[GU], Lu[GU];
    int64_t bu[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int idx = base + u * 128 + (int)threadIdx.x;
      const int q = idx / T;
      tt[u] = idx - q * T;
      bu[u] = b0 + q;
      const bool ok = idx < nit && bu[u] < B;
      const int64_t l = ok ? lengths[bu[u]] : -1;
      Lu[u] = ok ? (int)(l <= 0 ? 0 : (l < T ? l : T)) : -1;
      const float* aq = ws_al + (bu[u] * (int64_t)T + tt[u]) * K;
      const float* bq = ws_be + (bu[u] * (int64_t)T + tt[u] + 1) * K;
#pragma unroll
      for (int i = 0; i < K; ++i)
        xs[u][i] = (tt[u] < Lu[u] ? aq[i] : 0.f) + (tt[u] < Lu[u] - 1 ? bq[i] : 0.f);
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      if (Lu[u] < 0) continue;
      float* gq = gamma + (bu[u] * (int64_t)T + tt[u]) * K;
      if (tt[u] >= Lu[u]) {
#pragma unroll
        for (int i = 0; i < K; ++i) gq[i] = 0.f;
        continue;
      }
      float mx = NEG_INF;
#pragma unroll
      for (int i = 0; i < K; ++i) mx = fmaxf(mx, xs[u][i]);
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        xs[u][i] = mx == NEG_INF ? 0.f : fexp2(xs[u][i] - mx);
        sm += xs[u][i];
      }
#pragma unroll
      for (int i = 0; i < K; ++i) gq[i] = xs[u][i] / sm;
    }
  }
}

static int fb_lin_tier();

// the fused-gamma streaming kernel where its ring allows it and two workgroups per CU fit (VQHMM_FB_FUSE=0:
// the workspace + gamma-pass form; a test switch read per call, like VQHMM_FB_RES)
// NSQ = 2 unless VQHMM_FB_PAIR=0 (a test switch read per call; bit-identical to NSQ = 1)
static bool fb_pair_on() {
  const char* env = VQHMM_ENV("VQHMM_FB_PAIR");
  return !(env && env[0] == '0');
}
template <int K, bool W16>
static bool fb_fused_ok(int64_t T) {
  const char* env = VQHMM_ENV("VQHMM_FB_FUSE");
  if (env && env[0] == '0') return false;
  if constexpr (!FbStream<K, W16>::CAN_FUSE) return false;
  return T <= (1 << 20) && FbStream<K, W16>::lds_bytes(true, (int)T) <= 80 * 1024;
}

template <int K, bool W16>
static void fwdbwd_go(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                      int64_t T, float* gamma, float* logZ, float* ws, hipStream_t s) {
  const dim3 grid((unsigned)cdiv(B, Geo<K, W16>::SPW));
  static const int no_gamma = prof_env("VQHMM_FB_NOGAMMA");
  if constexpr (FbStream<K, W16>::CAN_FUSE) {
    if (fb_fused_ok<K, W16>(T)) {
      if (fb_pair_on()) {
        const dim3 grid2((unsigned)cdiv(B, 2 * Geo<K, W16>::SPW));
        fwdbwd_kernel<K, W16, true, 2><<<grid2, 512, 2 * FbStream<K, W16>::lds_bytes(true, (int)T), s>>>(
            log_pi, log_A, em, lengths, B, (int)T, gamma, logZ, ws, fb_lin_tier(), 0);
      } else {
        fwdbwd_kernel<K, W16, true><<<grid, 256, FbStream<K, W16>::lds_bytes(true, (int)T), s>>>(
            log_pi, log_A, em, lengths, B, (int)T, gamma, logZ, ws, fb_lin_tier(), 0);
      }
      return;
    }
  }
  fwdbwd_kernel<K, W16, false><<<grid, 128, FbStream<K, W16>::lds_bytes(false, (int)T), s>>>(
      log_pi, log_A, em, lengths, B, (int)T, gamma, logZ, ws, fb_lin_tier(), no_gamma);
}

// ------------------------------------------------- forward-backward, LDS-resident table
// For T up to ~550 the whole per-step table of a workgroup's SPW sequences fits in LDS, so
// HBM is read once: log_A and em are linearised once into m(i, j) = 2^((lg A + lg e) lg e)
// (the linear tier's table) and BOTH chains run on it, alpha upward and beta downward.
// Beta uses alpha's lane map at each data step d (map parity = d's parity; it reduces over
// the j axis, alpha over the i axis — both chains then alternate axes consistently), so one
// lane-major table [T/4][64 lanes][4 steps] serves both with one ds_read_b128 per 4 steps.
//
// One workgroup = 4 waves on SPW sequences, one per SIMD:
//   wave 0  alpha chain        wave 2  linearises chunks 0 .. hF-1 (upward), flushes alpha
//   wave 1  beta chain         wave 3  linearises chunks nch-1 .. hF (downward), flushes beta
// Iteration it (one LDS barrier each): alpha runs chunk it, beta data chunk nch-1-it; the
// helpers linearise the chunks the chains take next (global loads issued one iteration
// ahead) and flush what the chains produced in iteration it-1.  A chain value is stored for
// the other direction (LDS history) and gamma_t = softmax(al_t + be_t) is formed by whichever
// flush comes second: alpha's flush of t when be'[t+1] is already flushed (t/HC + (t+1)/HC >=
// nch), beta's flush when al_t is (t/HC + (t+1)/HC <= nch - 2); the few t between (= nch - 1)
// after the loop.  No workspace traffic: HBM sees log_A + em once and gamma once.
// The chains run the linear tier, with the log-tier / exact fallbacks reading the raw tables
// straight from global memory (rare path).
namespace {
constexpr int FR_HC = 16;  // steps per chunk of the resident kernel

template <int K>
struct FbRes {
  using Gm = Geo<K, false>;
  static constexpr int KP = Gm::KP, G = Gm::G, SPW = Gm::SPW, HC = FR_HC;
  static constexpr int VB = SPW * HC * KP;  // one chunk of chain values [SPW][HC][KP]
  static_assert(VB % 64 == 0, "flush covers whole wave passes");
  // LDS floats for a given T: table, two histories [SPW][HH][KP], vbuf [dir][2][VB], 4 flags
  __host__ __device__ static int hh(int T) { return ((T + HC - 1) / HC / 2 + 1) * HC; }
  static size_t lds_bytes(int T) {
    const size_t tp = (size_t)cdiv(T, HC) * HC;
    return (tp * 64 + 2 * (size_t)SPW * hh(T) * KP + 4 * (size_t)VB + 4) * sizeof(float);
  }
};
}  // namespace

template <int K>
__global__ __launch_bounds__(256) void fwdbwd_resident_kernel(const float* __restrict__ log_pi,
                                                              const float* __restrict__ log_A,
                                                              const float* __restrict__ em,
                                                              const int64_t* __restrict__ lengths, int64_t B, int T,
                                                              float* __restrict__ gamma, float* __restrict__ logZ,
                                                              int lin_tier, unsigned long long* __restrict__ prof) {
  using F = FbRes<K>;
  constexpr int KP = F::KP, G = F::G, SPW = F::SPW, HC = F::HC, VB = F::VB;
  extern __shared__ float4 smem_fr[];
  float* Mt = reinterpret_cast<float*>(smem_fr);
  const int nchT = (int)cdiv(T, HC), HH = F::hh(T);
  float* hist_a = Mt + (size_t)nchT * HC * 64;  // al_t at [q][t][state]
  float* hist_b = hist_a + SPW * HH * KP;       // be'[d] at [q][d - dbase][state]
  float* vb = hist_b + SPW * HH * KP;           // [dir][buf][VB]
  int* flags = reinterpret_cast<int*>(vb + 4 * VB);

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, grp = lane / G, g = lane % G;
  const int64_t b0 = (int64_t)blockIdx.x * SPW;
  const int64_t b = b0 + grp;
  const bool live = b < B;
  const int64_t Lr = live ? lengths[b] : 0;
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  int Lmax = L;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) Lmax = max(Lmax, __shfl_xor(Lmax, o));
  Lmax = __builtin_amdgcn_readfirstlane(Lmax);
  const int nch = (int)cdiv(Lmax, HC), hF = (nch + 1) / 2;
  const int dbase = ((nch - 1) / 2) * HC;  // first data step kept in hist_b
  const int jo = g % KP, ji = g / KP;
  // lane map per parity p of the data step: p = 0: (i, j) = (ji, jo); p = 1: (jo, ji)
  int aoff[2], ej[2];
  bool aok[2], eok[2], iok[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int i = p == 0 ? ji : jo, j = p == 0 ? jo : ji;
    aok[p] = i < K && j < K;
    eok[p] = j < K;
    iok[p] = i < K;
    aoff[p] = aok[p] ? i * K + j : 0;
    ej[p] = eok[p] ? j : 0;
  }
  const int64_t bc = live ? b : B - 1;  // dead groups read a valid sequence, never use it
  const float* Ab = log_A + bc * (int64_t)T * K * K;
  const float* Eb = em + bc * (int64_t)T * K;

  // ---- helpers: raw loads of a chunk into registers, then m = 2^((a + e) lg e) into the table
  float ra[HC], re[HC];
  auto load_raw = [&](int c) {
    if (c * HC + HC <= T) {  // whole chunk: one base per parity, immediate offsets
      const float* pa[2] = {Ab + (int64_t)c * HC * K * K + aoff[0], Ab + (int64_t)c * HC * K * K + aoff[1]};
      const float* pe[2] = {Eb + (int64_t)c * HC * K + ej[0], Eb + (int64_t)c * HC * K + ej[1]};
#pragma unroll
      for (int s = 0; s < HC; ++s) {
        const int p = s & 1;
        ra[s] = aok[p] ? pa[p][s * K * K] : NEG_INF;
        re[s] = eok[p] ? pe[p][s * K] : 0.f;
      }
    } else {
#pragma unroll
      for (int s = 0; s < HC; ++s) {
        const int p = s & 1;
        const int t = min(c * HC + s, T - 1);
        ra[s] = aok[p] ? Ab[(int64_t)t * K * K + aoff[p]] : NEG_INF;
        re[s] = eok[p] ? Eb[(int64_t)t * K + ej[p]] : 0.f;
      }
    }
  };
  auto linearise = [&](int c) {
#pragma unroll
    for (int q = 0; q < HC / 4; ++q) {
      float4 m;
      m.x = fexp2((ra[4 * q] + re[4 * q]) * LOG2E_F);
      m.y = fexp2((ra[4 * q + 1] + re[4 * q + 1]) * LOG2E_F);
      m.z = fexp2((ra[4 * q + 2] + re[4 * q + 2]) * LOG2E_F);
      m.w = fexp2((ra[4 * q + 3] + re[4 * q + 3]) * LOG2E_F);
      *reinterpret_cast<float4*>(&Mt[((size_t)(c * (HC / 4) + q) * 64 + lane) * 4]) = m;
    }
  };
  // raw log-domain values of a chunk for the fallback tiers (emx = max_j e, off the chain)
  float av[HC], dv[HC], xv[HC], mv[HC], ml[HC];
  auto read_raw = [&](int c, bool beta) {
#pragma unroll
    for (int s = 0; s < HC; ++s) {
      const int p = s & 1;
      const int t = min(c * HC + s, T - 1);
      const float a = aok[p] ? Ab[(int64_t)t * K * K + aoff[p]] : NEG_INF;
      const float e = eok[p] ? Eb[(int64_t)t * K + ej[p]] : 0.f;
      const float ein = eok[0] ? Eb[(int64_t)t * K + ej[0]] : NEG_INF;
      float emx = allred<KP, true>(ein, OpMax{});
      emx = emx == NEG_INF ? 0.f : emx;
      if (beta) {
        av[s] = (a + (e - emx)) * LOG2E_F;
      } else {
        av[s] = a * LOG2E_F;
        dv[s] = (e - emx) * LOG2E_F;
        xv[s] = emx;
      }
    }
  };
  auto read_table = [&](int c) {
#pragma unroll
    for (int q = 0; q < HC / 4; ++q) {
      const float4 m = *reinterpret_cast<const float4*>(&Mt[((size_t)(c * (HC / 4) + q) * 64 + lane) * 4]);
      ml[4 * q] = m.x;
      ml[4 * q + 1] = m.y;
      ml[4 * q + 2] = m.z;
      ml[4 * q + 3] = m.w;
    }
  };

  // ---- chains
  const float lp2 = jo < K ? log_pi[jo] * LOG2E_F : 0.f;
  float al = NEG_INF, be = 0.f, x = 0.f, sk = 0.f, lo = 1.f, hi = 1.f, rng = 0.f;
  double S2 = 0.0, SE = 0.0;

  auto alpha_chunk = [&](int c) {
    const int t0 = c * HC;
    float* vrow = vb + (c & 1) * VB + grp * HC * KP;
    // log tier (EXACT: max-shifted log-sum-exp; CHECK: some sequence ends inside the chunk)
    auto steps = [&](bool first, auto exact, auto check) {
      constexpr bool EXACT = decltype(exact)::value, CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = decltype(si)::value, p = s & 1;
        if (s == 0 && first) {
          al = (L > 0 && jo < K) ? lp2 + dv[0] : NEG_INF;
          mv[0] = 0.f;
          vrow[jo] = al;
          return;
        }
        const bool upd = !CHECK || t0 + s < L;
        const float v = al + av[s];
        float mus = 0.f;
        if constexpr (EXACT || s % FB_NORM == 0) {
          const float mu = allred<KP, p == 1>(al, OpMax{});
          mus = mu == NEG_INF ? 0.f : mu;
        }
        float nal;
        if constexpr (EXACT) {
          const float mm = fmaxf(allred<KP, p == 1>(v, OpMax{}), F32_LOWEST);
          const float sm = allred<KP, p == 1>(fexp2(v - mm), OpAdd{});
          nal = (mm + flog2(sm)) + (dv[s] - mus);
        } else {
          const float ls = flog2(allred<KP, p == 1>(fexp2(v), OpAdd{}));
          nal = ls + (dv[s] - mus);
          rng = fmaxf(rng, fabsf((eok[p] && upd) ? ls : 0.f));
        }
        mv[s] = upd ? mus : 0.f;
        if (upd) al = nal;
        vrow[s * KP + (p == 0 ? jo : ji)] = al;
      });
    };
    auto lin_steps = [&](bool first, float e0, auto check) {
      constexpr bool CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = decltype(si)::value, p = s & 1;
        if (s == 0 && first) {
          const float a0 = (L > 0 && jo < K) ? lp2 + e0 : NEG_INF;
          const float m0 = allred<KP, true>(a0, OpMax{});
          const float m0s = m0 == NEG_INF ? 0.f : m0;
          x = fexp2(a0 - m0s);
          sk = m0s;
          if (L > 0 && jo < K) lo = fminf(lo, x);
          vrow[jo] = x;
          return;
        }
        const bool upd = !CHECK || t0 + s < L;
        const float v = x * ml[s];
        int k = 0;
        if constexpr (s % FB_LNORM == FB_LNORM / 2) k = __builtin_amdgcn_frexp_expf(allred<KP, p == 1>(x, OpMax{}));
        float y = allred<KP, p == 1>(v, OpAdd{});
        if constexpr (s % FB_LNORM == FB_LNORM / 2) y = __builtin_amdgcn_ldexpf(y, -k);
        const bool chk = upd && eok[p];
        lo = chk ? fminf(lo, y) : lo;
        hi = chk ? fmaxf(hi, y) : hi;
        if (upd) {
          x = y;
          sk += (float)k;
        }
        vrow[s * KP + (p == 0 ? jo : ji)] = x;
      });
    };
    const float al_c = al;
    bool linear = false;
    if (lin_tier) {
      read_table(c);
      const float e0 = c == 0 && eok[0] ? Eb[ej[0]] * LOG2E_F : NEG_INF;
      lo = hi = 1.f;
      if (c > 0) {
        const float m = allred<KP, false>(al, OpMax{});
        const float ms = m == NEG_INF ? 0.f : m;
        x = fexp2(al - ms);
        sk = ms;
        if (t0 < L && ji < K) lo = fminf(lo, x);
      }
      if (__builtin_amdgcn_ballot_w64(t0 + HC > L) == 0) lin_steps(c == 0, e0, std::false_type{});
      else lin_steps(c == 0, e0, std::true_type{});
      linear = !__builtin_amdgcn_ballot_w64(lin_bad(lo, hi));
    }
    float dS2 = 0.f, dSE = 0.f;  // (one accumulation after the branch keeps S2 / SE in registers)
    if (linear) {
      if (t0 < L) {
        al = flog2(x);
        dS2 = sk;
      }
    } else {
      read_raw(c, false);
      al = al_c;
      rng = 0.f;
      steps(c == 0, std::false_type{}, std::true_type{});
      if (__builtin_amdgcn_ballot_w64(rng > FB_LIM)) {
        al = al_c;
        steps(c == 0, std::true_type{}, std::true_type{});
      }
#pragma unroll
      for (int s = 0; s < HC; ++s) xv[s] = t0 + s < L ? xv[s] : 0.f;
      dS2 = tree_sum<HC>(mv);
      dSE = tree_sum<HC>(xv);
    }
    S2 += (double)dS2;
    SE += (double)dSE;
    if (lane == 0) flags[c & 1] = linear;
  };

  // beta on data chunk k (data step d serves t = d - 1; map parity = d's parity)
  auto beta_chunk = [&](int k, int buf) {
    const int d0 = k * HC;
    float* vrow = vb + (2 + buf) * VB + grp * HC * KP;
    auto steps = [&](bool last, auto exact) {
      constexpr bool EXACT = decltype(exact)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = HC - 1 - decltype(si)::value, p = s & 1;
        if (s == 0 && last) return;  // t = -1
        const bool upd = d0 + s - 1 < L - 1;
        const float v = av[s] + be;
        float nus = 0.f;
        if constexpr (EXACT || s % FB_NORM == 0) {
          const float nu = allred<KP, p == 0>(be, OpMax{});
          nus = nu == NEG_INF ? 0.f : nu;
        }
        float nb;
        if constexpr (EXACT) {
          const float mm = fmaxf(allred<KP, p == 0>(v, OpMax{}), F32_LOWEST);
          const float sm = allred<KP, p == 0>(fexp2(v - mm), OpAdd{});
          nb = (mm + flog2(sm)) - nus;
        } else {
          const float ls = flog2(allred<KP, p == 0>(fexp2(v), OpAdd{}));
          nb = ls - nus;
          rng = fmaxf(rng, fabsf((iok[p] && upd) ? ls : 0.f));
        }
        if (upd) be = nb;
        vrow[s * KP + (p == 0 ? ji : jo)] = be;
      });
    };
    auto lin_steps = [&](bool last, auto check) {
      constexpr bool CHECK = decltype(check)::value;
      static_for<HC>([&](auto si) {
        constexpr int s = HC - 1 - decltype(si)::value, p = s & 1;
        if (s == 0 && last) return;
        const bool upd = !CHECK || d0 + s - 1 < L - 1;
        const float v = ml[s] * x;
        int kx = 0;
        if constexpr (s % FB_LNORM == FB_LNORM / 2) kx = __builtin_amdgcn_frexp_expf(allred<KP, p == 0>(x, OpMax{}));
        float y = allred<KP, p == 0>(v, OpAdd{});
        if constexpr (s % FB_LNORM == FB_LNORM / 2) y = __builtin_amdgcn_ldexpf(y, -kx);
        const bool chk = upd && iok[p];
        lo = chk ? fminf(lo, y) : lo;
        hi = chk ? fmaxf(hi, y) : hi;
        if (upd) x = y;
        vrow[s * KP + (p == 0 ? ji : jo)] = x;
      });
    };
    const float be_c = be;
    bool linear = false;
    if (lin_tier) {
      read_table(k);
      // state of data step d0 + HC (odd last step of the chunk: the j axis of map 1 = outer)
      const float m = allred<KP, false>(be, OpMax{});
      x = fexp2(be - (m == NEG_INF ? 0.f : m));
      lo = hi = 1.f;
      if (d0 + HC - 1 < L - 1 && ji < K) lo = fminf(lo, x);
      const bool full = d0 + HC <= L;  // every step of the chunk is live for this sequence
      if (__builtin_amdgcn_ballot_w64(!full) == 0) lin_steps(k == 0, std::false_type{});
      else lin_steps(k == 0, std::true_type{});
      linear = !__builtin_amdgcn_ballot_w64(lin_bad(lo, hi));
    }
    if (linear) {
      be = flog2(x);
    } else {
      read_raw(k, true);
      be = be_c;
      rng = 0.f;
      steps(k == 0, std::false_type{});
      if (__builtin_amdgcn_ballot_w64(rng > FB_LIM)) {
        be = be_c;
        steps(k == 0, std::true_type{});
      }
    }
    if (lane == 0) flags[2 + buf] = linear;
  };

  // ---- flushes (helpers): chain values -> history and/or gamma
  auto seqlen = [&](int q) {
    const int64_t bq = b0 + q;
    if (bq >= B) return -1;
    const int64_t l = lengths[bq];
    return (int)(l <= 0 ? 0 : (l < T ? l : T));
  };
  // sequence lengths of the flush lanes (pass r covers sequence (r * 64 + lane) / (HC * KP))
  int Lfl[VB / 64];
#pragma unroll
  for (int r = 0; r < VB / 64; ++r) Lfl[r] = seqlen((r * 64 + lane) / (HC * KP));
  // softmax over the KP-lane state group of lanes idx % KP (padding states masked)
  auto store_gamma = [&](int q, int t, int j, float xs, bool own) {
    const float xm = (j < K) ? xs : NEG_INF;
    const float mx = allred<KP, true>(xm, OpMax{});
    const float ex = (j < K && mx != NEG_INF) ? fexp2(xm - mx) : 0.f;
    const float sm = allred<KP, true>(ex, OpAdd{});
    if (own && j < K) gamma[((b0 + q) * (int64_t)T + t) * K + j] = ex * __builtin_amdgcn_rcpf(sm);
  };
  auto flush_alpha = [&](int c) {
    const bool lin = flags[c & 1] != 0;
    const float* src = vb + (c & 1) * VB;
#pragma unroll
    for (int r = 0; r < VB / 64; ++r) {
      const int idx = r * 64 + lane;
      const int q = idx / (HC * KP), rr = idx - q * (HC * KP), s = rr / KP, j = rr - s * KP;
      const int t = c * HC + s;
      const float v = lin ? flog2(src[idx]) : src[idx];
      if (t < HH) hist_a[(q * HH + t) * KP + j] = v;
      const int Lq = Lfl[r];
      const bool ok = Lq >= 0 && t < T;
      const bool own = ok && (t >= Lq - 1 || t / HC + (t + 1) / HC >= nch);
      const bool past = ok && t >= Lq;  // gamma_t = 0 past the sequence
      float xs = v;
      if (own && t < Lq - 1) xs += hist_b[(q * HH + (t + 1 - dbase)) * KP + j];
      store_gamma(q, t, j, xs, own && !past);
      if (past && j < K) gamma[((b0 + q) * (int64_t)T + t) * K + j] = 0.f;
    }
  };
  auto flush_beta = [&](int k, int buf) {
    const bool lin = flags[2 + buf] != 0;
    const float* src = vb + (2 + buf) * VB;
#pragma unroll
    for (int r = 0; r < VB / 64; ++r) {
      const int idx = r * 64 + lane;
      const int q = idx / (HC * KP), rr = idx - q * (HC * KP), s = rr / KP, j = rr - s * KP;
      const int d = k * HC + s, t = d - 1;
      const float v = lin ? flog2(src[idx]) : src[idx];
      if (d >= dbase && d - dbase < HH) hist_b[(q * HH + (d - dbase)) * KP + j] = v;
      const int Lq = Lfl[r];
      const bool own = Lq >= 0 && t >= 0 && t < Lq - 1 && t / HC + d / HC <= nch - 2;
      const float xs = own ? hist_a[(q * HH + t) * KP + j] + v : 0.f;
      store_gamma(q, t, j, xs, own);
    }
  };

  // ---- schedule
  if (wave == 2 && nch > 0) {
    load_raw(0);
    linearise(0);
    if (1 < hF) load_raw(1);
  } else if (wave == 3 && nch - 1 >= hF) {
    load_raw(nch - 1);
    linearise(nch - 1);
    if (nch - 2 >= hF) load_raw(nch - 2);
  }
  lds_barrier();
  unsigned long long pt0 = 0, pbusy = 0, plin = 0;  // (VQHMM_FB_PROF: per-wave cycle counts)
  if (prof) pt0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it <= nch; ++it) {
    unsigned long long ta = 0, tb = 0;
    if (prof) ta = __builtin_amdgcn_s_memtime();
    if (wave == 0) {
      if (it < nch) alpha_chunk(it);
    } else if (wave == 1) {
      if (it < nch) beta_chunk(nch - 1 - it, it & 1);
    } else if (wave == 2) {
      if (it + 1 < hF) {
        linearise(it + 1);
        if (it + 2 < hF) load_raw(it + 2);
      }
      if (prof) tb = __builtin_amdgcn_s_memtime();
      if (it >= 1) flush_alpha(it - 1);
    } else {
      const int c = nch - 2 - it;
      if (c >= hF) {
        linearise(c);
        if (c - 1 >= hF) load_raw(c - 1);
      }
      if (prof) tb = __builtin_amdgcn_s_memtime();
      if (it >= 1) flush_beta(nch - it, (it - 1) & 1);
    }
    if (prof) {
      __builtin_amdgcn_s_waitcnt(0);
      const unsigned long long tc = __builtin_amdgcn_s_memtime();
      pbusy += tc - ta;
      plin += tb ? tb - ta : 0;
    }
    lds_barrier();
  }
  if (prof && lane == 0) {
    unsigned long long* o = prof + ((size_t)blockIdx.x * 4 + wave) * 4;
    o[0] = __builtin_amdgcn_s_memtime() - pt0;
    o[1] = pbusy;
    o[2] = plin;
    o[3] = (unsigned long long)nch;
  }

  if (wave == 0) {  // logZ from the state axis held after step L-1 (even t: inner)
    const int tl = L - 1;
    const bool held_inner = (tl <= 0) || ((tl & 1) == 0);
    const int st = held_inner ? jo : ji;
    const float x0 = st < K ? al : NEG_INF;
    const float mx = held_inner ? allred<KP, true>(x0, OpMax{}) : allred<KP, false>(x0, OpMax{});
    const float mxs = fmaxf(mx, F32_LOWEST);
    const float ex = fexp2(x0 - mxs);
    const float sx = held_inner ? allred<KP, true>(ex, OpAdd{}) : allred<KP, false>(ex, OpAdd{});
    if (live && g == 0)
      logZ[b] = L > 0 ? (float)(LN2_D * (S2 + (double)mxs + (double)flog2(sx)) + SE)
                      : __builtin_bit_cast(float, 0x7fc00000u);
  } else if (wave == 2) {  // the steps between the two flush rules: t/HC + (t+1)/HC == nch - 1
    const int tb = max(((nch - 1) / 2) * HC - 1, 0);
    for (int idx = lane; idx < SPW * 2 * HC * KP; idx += 64) {  // wave-uniform trip count
      const int q = idx / (2 * HC * KP), rr = idx - q * (2 * HC * KP), s = rr / KP, j = rr - s * KP;
      const int t = tb + s;
      const int Lq = seqlen(q);
      const bool own = Lq >= 0 && t < Lq - 1 && t / HC + (t + 1) / HC == nch - 1;
      const float xs = own ? hist_a[(q * HH + t) * KP + j] + hist_b[(q * HH + (t + 1 - dbase)) * KP + j] : 0.f;
      store_gamma(q, t, j, xs, own);
    }
  } else if (wave == 3) {  // steps no chain reached: t >= nch * HC
    const int t0 = nch * HC, nt = T - t0;
    for (int64_t idx = lane; idx < (int64_t)SPW * nt * K; idx += 64) {
      const int q = (int)(idx / ((int64_t)nt * K));
      const int64_t rr = idx - (int64_t)q * nt * K;
      if (b0 + q < B) gamma[((b0 + q) * (int64_t)T + t0) * K + rr] = 0.f;
    }
  }
}

static int fb_lin_tier() {  // VQHMM_FB_LIN=0: log tier only (A/B switch)
  static const int lin = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_FB_LIN");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return lin;
}

// the resident kernel when its LDS fits (VQHMM_FB_RES=0: always the streaming kernel)
// CU count and LDS bytes per workgroup of the current device, queried once per device
// (the kernel choice below sizes one round of resident workgroups from them).
struct DevShape {
  int cus = 0;
  size_t lds = 0;
};
static DevShape dev_shape() {
  static DevShape cache[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  DevShape& d = cache[dev];
  if (d.cus == 0) {
    int cus = 0, lds = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || lds <= 0)
      lds = 64 * 1024;
    d.lds = (size_t)lds;
    d.cus = cus;
  }
  return d;
}

static bool fwdbwd_resident_ok(int64_t B, int64_t K, int64_t T) {
  // VQHMM_FB_RES=0 forces the streaming kernel: a test switch, read per call because the tests
  // run both kernels in one process
  const char* env = VQHMM_ENV("VQHMM_FB_RES");
  if ((env && env[0] == '0') || K < 1 || K > 8 || T > 4096) return false;
  const int kp = K <= 2 ? 2 : K <= 4 ? 4 : 8;
  const size_t bytes = kp == 2 ? FbRes<2>::lds_bytes((int)T) : kp == 4 ? FbRes<4>::lds_bytes((int)T)
                                                                     : FbRes<8>::lds_bytes((int)T);
  const DevShape dv = dev_shape();
  if (bytes > dv.lds) return false;
  // one round of workgroups only: a second round doubles the chain time, and the streaming
  // kernel (two reads of the table, twice the workgroups per CU) is then faster
  const int64_t spw = 64 / (kp * kp), per_cu = (int64_t)(dv.lds / bytes);
  return cdiv(B, spw) <= (int64_t)dv.cus * per_cu;
}

template <int K>
static void fwdbwd_res_go(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                          int64_t T, float* gamma, float* logZ, void* ws, hipStream_t s) {
  const dim3 grid((unsigned)cdiv(B, FbRes<K>::SPW));
  static const bool prof = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_FB_PROF");  // diagnostic: per-wave cycle counts into the workspace
    return e && e[0] == '1';
  }();
  fwdbwd_resident_kernel<K><<<grid, 256, FbRes<K>::lds_bytes((int)T), s>>>(
      log_pi, log_A, em, lengths, B, (int)T, gamma, logZ, fb_lin_tier(), prof ? (unsigned long long*)ws : nullptr);
}

size_t fwdbwd_ws_bytes(int64_t B, int64_t T, int64_t K) { return 2 * (size_t)B * T * K * sizeof(float); }

int launch_fwdbwd(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                  int64_t T, int64_t K, float* gamma, float* logZ, void* ws, size_t ws_bytes, hipStream_t s) {
  if (B == 0) return VQHMM_OK;
  if (K < 1 || !hmm_generic_supported(K) || T < 1 || T > (1 << 28)) return VQHMM_EUNSUPPORTED;
  if (!ws || ws_bytes < fwdbwd_ws_bytes(B, T, K)) return VQHMM_EWORKSPACE;
  if (K > 32) return launch_fwdbwd_generic(log_pi, log_A, em, lengths, B, T, K, gamma, logZ, ws, s);
  const bool w16 = aligned16(log_A) && aligned16(em);
  float* w = (float*)ws;
  if (K > 8) return launch_fwdbwd_wide(log_pi, log_A, em, lengths, B, T, K, gamma, logZ, w, s);
  if (fwdbwd_seg_ok(B, T, K)) return launch_fwdbwd_seg(log_pi, log_A, em, lengths, B, T, K, gamma, logZ, w, s);
  if (fwdbwd_resident_ok(B, K, T)) {
    switch (K) {
      case 1: fwdbwd_res_go<1>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      case 2: fwdbwd_res_go<2>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      case 3: fwdbwd_res_go<3>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      case 4: fwdbwd_res_go<4>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      case 5: fwdbwd_res_go<5>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      case 6: fwdbwd_res_go<6>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      case 7: fwdbwd_res_go<7>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
      default: fwdbwd_res_go<8>(log_pi, log_A, em, lengths, B, T, gamma, logZ, ws, s); break;
    }
    VQHMM_LAUNCH_CHECK();
    return VQHMM_OK;
  }
  switch (K) {
    case 1: fwdbwd_go<1, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s); break;
    case 2: fwdbwd_go<2, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s); break;
    case 3: fwdbwd_go<3, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s); break;
    case 4:
      if (w16) fwdbwd_go<4, true>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s);
      else fwdbwd_go<4, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s);
      break;
    case 5: fwdbwd_go<5, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s); break;
    case 6: fwdbwd_go<6, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s); break;
    case 7: fwdbwd_go<7, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s); break;
    default:
      if (w16) fwdbwd_go<8, true>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s);
      else fwdbwd_go<8, false>(log_pi, log_A, em, lengths, B, T, gamma, logZ, w, s);
      break;
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
