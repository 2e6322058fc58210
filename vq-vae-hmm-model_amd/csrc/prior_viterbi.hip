// Fused Prior.forward -> Viterbi (Prior VQ_VAE_HMM_fixed.py:53-71, recursion A16):
// the MAP path over transition tables that are computed on the chip from u and never written to HBM.
// The unfused path writes log_A (B, T, K, K) with prior.hip and reads it back in viterbi_kernel:
// 4K^2 + 4K^2 bytes per position (512 B at K = 8) against 4U here, the u row.
//
// One workgroup = NW waves (8 for trans_hidden <= 128: two per SIMD) and NU "units" (one unit = the
// SPW sequences one Viterbi wave carries in its KP^2-lane groups, hmm_lanes.h).  Per chunk of HC steps:
//   1. every wave computes MLP tiles (prior_tile.h: the same MFMA sequence and row log_softmax as
//      prior.hip, so the tables are bit-identical to model.prior(u)'s) straight into the units'
//      LDS chunk slot, in viterbi_kernel's slot layout [SPW][HC][K][K]; the emissions of the chunk go
//      beside them ([SPW][HC][K]); u and em for the NEXT chunk are already in flight in registers;
//   2. one LDS barrier;
//   3. waves 0 .. NU-1 run the unit's max-plus chain on the slot (viterbi_kernel's step: same
//      fp32 order, ballot backpointers), while the other waves go on to the next chunk's tiles
//      (on the same SIMD, so a chain's latency-bound steps sit beside another wave's MFMAs).
// Slots are double-buffered per unit, so a chunk's tables are overwritten only after the next
// barrier.  After the last chunk every chain wave backtraces its unit alone, staging the mask
// stream through its own (now idle) slot pair.
// Cost: the MLP is 2(U + KK) TH flops per position on f32 MFMA (17.4 kflop at K = 8, TH = 128), the
// chain ~100 cycles per step; the kernel is MFMA-bound (tools/infer_bench.py).
// Bit-exact contract: path and score equal vqhmm_viterbi_f32 on vqhmm_prior_f32's log_A (and so
// oracle_viterbi_f32 on that table).
#include "hmm_lanes.h"
#include "prior_tile.h"

#include <stdlib.h>

namespace vqhmm {

namespace {
// viterbi_kernel's slot geometry (hmm_lanes.h Geo) with a free chunk length HC
template <int K, int HC_>
struct PGeo {
  static constexpr int HC = HC_;
  static constexpr int KP = Geo<K, false>::KP, G = KP * KP, SPW = 64 / G;
  static constexpr int AS = HC * K * K, ES = HC * K, SLOT = SPW * (AS + ES);
};

template <int K, int NW, int HC>
struct PVGeo {
  using Gm = PGeo<K, HC>;
  static constexpr int NU = Gm::SPW > 1 ? 1 : 4;           // chain waves per workgroup
  static constexpr int TPC = Gm::SPW * HC / 16;              // MLP tiles per unit per chunk
  static constexpr int NT = NU * TPC;                        // MLP tiles per chunk
  static constexpr int TPW = (NT + NW - 1) / NW;             // per wave
  static constexpr int NE = NU * Gm::SPW * HC * K;           // emissions per chunk
  static constexpr int EPT = (NE + 64 * NW - 1) / (64 * NW); // per thread
};

template <int K, int HB, int NW, int HC>
struct PVLds {
  PriorW<HB, prior_kb(K)> w;
  float zS[NW][16 * PriorW<HB, prior_kb(K)>::LDZ];
  float slot[PVGeo<K, NW, HC>::NU][2][PGeo<K, HC>::SLOT];
  int lmax[NW];
};
}  // namespace

template <int K, int HB, int NW, int HC>
__global__ __launch_bounds__(NW * 64) void prior_viterbi_kernel(PriorArgs p, const float* __restrict__ log_pi,
                                                            const float* __restrict__ em,
                                                            const int64_t* __restrict__ lengths,
                                                            int32_t* __restrict__ path, float* __restrict__ score,
                                                            uint2* __restrict__ masks, int mode) {
  constexpr int KB = prior_kb(K);
  using Gm = PGeo<K, HC>;
  using PG = PVGeo<K, NW, HC>;
  using S = PVLds<K, HB, NW, HC>;
  constexpr int KP = Gm::KP, G = Gm::G, SPW = Gm::SPW, NU = PG::NU, NTH = NW * 64;
  constexpr int LDZ = PriorW<HB, KB>::LDZ;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform: the chain branch is scalar
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int64_t B = p.B;
  const int T = p.T, U = p.U;
  prior_stage_weights<HB, KB>(sh.w, p.W1, p.b1, p.W2, K, U, tid, NTH);
  f32x4 b2f[KB];
  prior_b2_frags<KB>(b2f, p.b2, K * K, lg4);

  // ---- chain state (waves < NU): unit blockIdx.x * NU + wave
  const int64_t unit = (int64_t)blockIdx.x * NU + wave;
  const int64_t b0 = unit * SPW;
  const bool chain = wave < NU && b0 < B;
  const int grp = lane / G, g = lane % G;
  const int64_t b = b0 + grp;
  const int64_t Lr = (chain && b < B) ? lengths[b] : 0;
  const int L = (int)(Lr <= 0 ? 0 : (Lr < T ? Lr : T));
  const int i0 = g % KP;
  const float lp = i0 < K ? log_pi[i0] : 0.f;
  int Lmax = L, Lmin = L;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    Lmax = max(Lmax, __shfl_xor(Lmax, o));
    Lmin = min(Lmin, __shfl_xor(Lmin, o));
  }
  Lmin = __builtin_amdgcn_readfirstlane(Lmin);
  if (lane == 0) sh.lmax[wave] = Lmax;
  __syncthreads();  // weights staged, lengths published
  int lwg = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) lwg = max(lwg, sh.lmax[w]);
  const int nchunks = (int)cdiv(lwg, HC);
  const int Tr = (int)cdiv(T, 64) * 64;
  uint2* wmask = masks + (size_t)unit * Tr;
  const LaneMap<K, false, Gm> lm(grp, g);

  // ---- producer side: this wave's tiles (tile tt = wave + NW k over [NU][SPW][HC/16]) and emissions
  auto tile_seq = [&](int tt, int& uu, int& q, int& h) {
    uu = tt / PG::TPC;
    const int r = tt - uu * PG::TPC;
    q = r / (HC / 16);
    h = r - q * (HC / 16);
  };
  auto load_u = [&](int c, float* ub) {
#pragma unroll
    for (int k = 0; k < PG::TPW; ++k) {
      const int tt = wave + NW * k;
      int uu, q, h;
      tile_seq(tt, uu, q, h);
      const int64_t bt = ((int64_t)blockIdx.x * NU + uu) * SPW + q;
      const int t = c * HC + 16 * h + l16;
      ub[k] = (tt < PG::NT && bt < B && t < T && lg4 < U)
                  ? p.u[bt * (int64_t)U * T + lg4 * p.u_sc + (int64_t)t * p.u_st]
                  : 0.f;
    }
  };
  auto load_e = [&](int c, float* ev) {
#pragma unroll
    for (int k = 0; k < PG::EPT; ++k) {
      const int e = tid + NTH * k;
      const int j = e % K, s = (e / K) % HC, q = (e / (K * HC)) % SPW, uu = e / (K * HC * SPW);
      int64_t bt = ((int64_t)blockIdx.x * NU + uu) * SPW + q;
      bt = bt < B ? bt : B - 1;
      int t = c * HC + s;
      t = t < T ? t : T - 1;
      ev[k] = e < PG::NE ? em[(bt * T + t) * K + j] : 0.f;
    }
  };
  float* zS = sh.zS[wave];
  auto produce = [&](int c, const float* ub, const float* ev) {
    const int par = c & 1;
#pragma unroll
    for (int k = 0; k < PG::TPW; ++k) {
      const int tt = wave + NW * k;
      int uu, q, h;
      tile_seq(tt, uu, q, h);
      const int64_t bt = ((int64_t)blockIdx.x * NU + uu) * SPW + q;
      if (tt >= PG::NT || bt >= B) continue;  // wave-uniform
      prior_tile<HB, KB>(sh.w, b2f, ub[k], l16, lg4, zS);
      __builtin_amdgcn_wave_barrier();
      float* dst = &sh.slot[uu][par][q * Gm::AS + 16 * h * K * K];
      for (int idx = lane; idx < 16 * K; idx += 64) {
        const int pos = idx / K, i = idx - pos * K;
        prior_row_lsm(&zS[pos * LDZ + i * K], K, dst + pos * K * K + i * K);
      }
      __builtin_amdgcn_wave_barrier();  // zS is rewritten by the next tile
    }
#pragma unroll
    for (int k = 0; k < PG::EPT; ++k) {
      const int e = tid + NTH * k;
      if (e >= PG::NE) continue;
      const int j = e % K, s = (e / K) % HC, q = (e / (K * HC)) % SPW, uu = e / (K * HC * SPW);
      sh.slot[uu][par][SPW * Gm::AS + q * Gm::ES + s * K + j] = ev[k];
    }
  };

  // ---- consumer side: viterbi_kernel's chunk step on the slot
  float d = NEG_INF;
  uint32_t mlo = 0, mhi = 0;
  constexpr int HBAT = 8;  // ballots per hazard-padded writelane batch
  auto run_chunk = [&](const float* av, const float* ev, int t0, bool first, auto check) {
    constexpr bool CHECK = decltype(check)::value;
    static_for<HC / 8>([&](auto hi) {
      constexpr int hh = decltype(hi)::value;
      uint64_t bal[HBAT];
      static_for<HBAT>([&](auto si) {
        constexpr int s = hh * HBAT + decltype(si)::value, pp = s & 1;
        if (s == 0 && first) {
          d = (L > 0 && i0 < K) ? lp + ev[0] : NEG_INF;
          bal[0] = 0;
          return;
        }
        const float v = d + av[s];
        const float m = pp == 0 ? allred<KP, false>(v, OpMax{}) : allred<KP, true>(v, OpMax{});
        bal[s - hh * HBAT] = __builtin_amdgcn_ballot_w64(v == m);
        if (!CHECK || t0 + s < L) d = m + ev[s];
      });
      writelane8<hh * HBAT>(mlo, mhi, bal);
    });
  };

  float ubn[PG::TPW], ebn[PG::EPT];
  if (nchunks > 0) {
    load_u(0, ubn);
    load_e(0, ebn);
  }
  for (int c = 0; c < nchunks; ++c) {
    float ubc[PG::TPW], ebc[PG::EPT];
#pragma unroll
    for (int k = 0; k < PG::TPW; ++k) ubc[k] = ubn[k];
#pragma unroll
    for (int k = 0; k < PG::EPT; ++k) ebc[k] = ebn[k];
    if (c + 1 < nchunks) {  // next chunk's operands in flight across this chunk's work
      load_u(c + 1, ubn);
      load_e(c + 1, ebn);
    }
    if (!(mode & 2)) produce(c, ubc, ebc);
    lds_barrier();
    if (chain && !(mode & 1)) {
      const float* sl = sh.slot[wave][c & 1];
      float av[HC], ev[HC];
#pragma unroll
      for (int s = 0; s < HC; ++s) {
        const int pp = s & 1;  // parity of t (t0 even)
        av[s] = lm.a_ok[pp] ? sl[lm.a_off[pp] + s * K * K] : NEG_INF;
        ev[s] = lm.e_ok[pp] ? sl[lm.e_off[pp] + s * K] : 0.f;
      }
      const int t0 = c * HC;
      if (t0 + HC <= Lmin) run_chunk(av, ev, t0, c == 0, std::false_type{});
      else run_chunk(av, ev, t0, c == 0, std::true_type{});
      if (lane < HC) wmask[t0 + lane] = make_uint2(mlo, mhi);  // masks of steps t0 .. t0 + HC - 1
    }
  }
  if (!chain) return;

  // ---- final state and backtrace (viterbi_kernel's, one wave on its own unit)
  const int tl = L - 1;
  const bool held_inner = (tl <= 0) || ((tl & 1) == 0);
  const int st = held_inner ? g % KP : g / KP;
  float best = (st < K) ? d : NEG_INF;
  int arg = st;
  if (held_inner) allargmax<KP, true>(best, arg); else allargmax<KP, false>(best, arg);

  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  constexpr int WT = (2 * Gm::SLOT * 4 / 8) / 64 * 64;
  static_assert(WT >= 64, "slot pair too small for a mask window");
  uint2* wl = reinterpret_cast<uint2*>(&sh.slot[wave][0][0]);
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
    int state = sq;
    for (int w0 = ((Lq - 1) / WT) * WT; Lq > 1 && w0 >= 0; w0 -= WT) {
      const int lo = max(w0, 1), hi = min(w0 + WT - 1, Lq - 1);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      const int nblk = (hi - w0) / 64 + 1;
      for (int k = 0; k < 2 * nblk; ++k)  // 64 dwords per instruction
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(wmask + w0) + k * 64 + lane,
                                         (__attribute__((address_space(3))) void*)(reinterpret_cast<uint32_t*>(wl) +
                                                                                   k * 64),
                                         4, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      const int n = hi - lo + 1;
      const int cl = (int)cdiv(n, 64);
      const int clo = lo + lane * cl, chi = min(clo + cl - 1, hi);
      uint32_t flo = 0x03020100u, fhi = 0x07060504u;
      for (int t = chi; t >= clo; --t) {
        const uint2 mm = wl[t - w0];
        const uint2 mp = bp_map<K>(mm.x, mm.y, q, t & 1);
        flo = perm_bytes(mp, flo);
        fhi = perm_bytes(mp, fhi);
      }
      int ecur = state, mine = 0;
      for (int cc = 63; cc >= 0; --cc) {
        const int slo = lo + cc * cl;
        if (slo > hi) continue;
        mine = lane == cc ? ecur : mine;
        const uint32_t xl = __builtin_amdgcn_readlane((int)flo, cc), xh = __builtin_amdgcn_readlane((int)fhi, cc);
        ecur = (int)((ecur < 4 ? (xl >> (8 * ecur)) : (xh >> (8 * (ecur - 4)))) & 0xFFu);
      }
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

bool prior_viterbi_supported(const PriorArgs& p) {
  return p.K >= 1 && p.K <= 8 && p.U >= 1 && p.U <= 4 && (p.TH == 64 || p.TH == 128 || p.TH == 256);
}

// profiling switch (VQHMM_PV_MODE: 1 = no chain, 2 = no tables; results then invalid)
static int pv_mode() {
  static const int m = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_PV_MODE");
    return e ? atoi(e) : 0;
  }();
  return m;
}

// TH <= 128: 8 waves (two per SIMD: one wave's chain runs beside the other's MFMA tiles), 32-step
// chunks (8 tiles per chunk); TH = 256: the weights leave room for 4 waves and 16-step chunks only.
template <int K, int HB>
static int launch_pv(const PriorArgs& p, const float* log_pi, const float* em, const int64_t* lengths, int32_t* path,
                     float* score, void* ws, hipStream_t s) {
  constexpr int NW = HB <= 8 ? 8 : 4, HC = HB <= 8 ? 32 : 16;
  constexpr int NU = PVGeo<K, NW, HC>::NU, SPW = PGeo<K, HC>::SPW;
  static_assert(sizeof(PVLds<K, HB, NW, HC>) <= 160 * 1024, "LDS");
  const int64_t units = cdiv(p.B, SPW);
  const dim3 grid((unsigned)cdiv(units, NU));
  prior_viterbi_kernel<K, HB, NW, HC><<<grid, NW * 64, sizeof(PVLds<K, HB, NW, HC>), s>>>(p, log_pi, em, lengths,
                                                                                          path, score, (uint2*)ws, pv_mode());
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

template <int HB>
static int launch_pv_k(const PriorArgs& p, const float* log_pi, const float* em, const int64_t* lengths,
                       int32_t* path, float* score, void* ws, hipStream_t s) {
  switch (p.K) {
    case 1: return launch_pv<1, HB>(p, log_pi, em, lengths, path, score, ws, s);
    case 2: return launch_pv<2, HB>(p, log_pi, em, lengths, path, score, ws, s);
    case 3: return launch_pv<3, HB>(p, log_pi, em, lengths, path, score, ws, s);
    case 4: return launch_pv<4, HB>(p, log_pi, em, lengths, path, score, ws, s);
    case 5: return launch_pv<5, HB>(p, log_pi, em, lengths, path, score, ws, s);
    case 6: return launch_pv<6, HB>(p, log_pi, em, lengths, path, score, ws, s);
    case 7: return launch_pv<7, HB>(p, log_pi, em, lengths, path, score, ws, s);
    default: return launch_pv<8, HB>(p, log_pi, em, lengths, path, score, ws, s);
  }
}

// p.log_A unused; log_pi = log_softmax(log_prior) already on the device; ws = viterbi_ws_bytes(B, T, K)
int launch_prior_viterbi(const PriorArgs& p, const float* log_pi, const float* em, const int64_t* lengths,
                         int32_t* path, float* score, void* ws, size_t ws_bytes, hipStream_t s) {
  if (!prior_viterbi_supported(p)) return VQHMM_EUNSUPPORTED;
  if (p.B == 0) return VQHMM_OK;
  if (p.T < 1) return VQHMM_EUNSUPPORTED;
  if (!ws || ws_bytes < viterbi_ws_bytes(p.B, p.T, p.K)) return VQHMM_EWORKSPACE;
  switch (p.TH) {
    case 64: return launch_pv_k<4>(p, log_pi, em, lengths, path, score, ws, s);
    case 128: return launch_pv_k<8>(p, log_pi, em, lengths, path, score, ws, s);
    default: return launch_pv_k<16>(p, log_pi, em, lengths, path, score, ws, s);
  }
}

}  // namespace vqhmm
