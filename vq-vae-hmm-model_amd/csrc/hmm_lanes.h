// Lane-group machinery of the K <= 8 HMM kernels (hmm.hip, prior_viterbi.hip): the (i, j) <-> lane
// maps, DPP / permlane reductions, LDS-ring chunk geometry and DMA staging, and the Viterbi
// backpointer-ballot helpers.  See hmm.hip's header comment for the design.
#pragma once
#include <type_traits>

#include "kernels.h"

namespace vqhmm {

constexpr float NEG_INF = -__builtin_inff();
template <int K, bool W16>
struct Geo {
  // steps per staged chunk: a chunk's LDS-DMA instructions x ring depth must
  // stay under vmcnt's 63 outstanding (more wraps the counter), so the
  // many-sequences-per-wave small-K maps and 4-byte K = 8 staging use half chunks
  static constexpr int HC = W16 ? 32 : (K <= 4 || K == 8) ? 16 : 32;
  static constexpr int KP = K <= 2 ? 2 : K <= 4 ? 4 : 8;
  static constexpr int G = KP * KP;     // lanes per sequence
  static constexpr int SPW = 64 / G;    // sequences per wave
  static constexpr int AS = HC * K * K;  // floats of log_A per sequence per chunk
  static constexpr int ES = HC * K;      // floats of em per sequence per chunk
  static constexpr int SLOT = SPW * (AS + ES);
};

// glds instructions per chunk and ring depth: R chunks of NI instructions can
// be outstanding at once (the wait leaves R - 1 in flight); vmcnt counts to 63
template <int K, bool W16>
struct Ring {
  static constexpr int U = W16 ? 4 : 1;  // floats per lane per instruction
  static constexpr int NI = Geo<K, W16>::SLOT / (64 * U);
  static_assert(Geo<K, W16>::SLOT % (64 * U) == 0, "slot must be whole wave-instructions");
  static constexpr int RD = 60 / NI;
  static constexpr int R = RD > 4 ? 4 : RD;
  static_assert(R >= 2, "chunk too large for a pipelined ring");
  static constexpr int WAIT = NI * (R - 1);
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1
template <int I, int N>
struct SFor {
  template <typename F>
  __device__ __forceinline__ static void run(F& f) {
    f(std::integral_constant<int, I>{});
    SFor<I + 1, N>::run(f);
  }
};
template <int N>
struct SFor<N, N> {
  template <typename F>
  __device__ __forceinline__ static void run(F&) {}
};
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  SFor<0, N>::run(f);
}

// ---------------------------------------------------------------- lane exchanges
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_XOR1 = 0xB1;          // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;          // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141;  // l -> 7 - l within 8 lanes
constexpr int DPP_ROR4 = 0x124;         // row_ror:4 (16-lane rows)
constexpr int DPP_ROR8 = 0x128;         // row_ror:8

struct OpMax {
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
struct OpAdd {
  __device__ float operator()(float a, float b) const { return a + b; }
};

// all-reduce over the KP lanes of one axis of a sequence's lane group:
// INNER = lanes g % KP (stride 1), else lanes g / KP (stride KP)
template <int KP, bool INNER, typename Op>
__device__ __forceinline__ float allred(float v, Op op) {
  if constexpr (KP == 2) {
    v = op(v, dpp<INNER ? DPP_XOR1 : DPP_XOR2>(v));
  } else if constexpr (KP == 4) {
    if constexpr (INNER) {
      v = op(v, dpp<DPP_XOR1>(v));
      v = op(v, dpp<DPP_XOR2>(v));
    } else {  // cosets {l, l+4, l+8, l+12} of a 16-lane row: two rotations
      v = op(v, dpp<DPP_ROR4>(v));
      v = op(v, dpp<DPP_ROR8>(v));
    }
  } else {
    if constexpr (INNER) {
      v = op(v, dpp<DPP_XOR1>(v));
      v = op(v, dpp<DPP_XOR2>(v));
      v = op(v, dpp<DPP_HALF_MIRROR>(v));
    } else {
      v = op(v, dpp<DPP_ROR8>(v));
      const float2 r16 = pair16(v);
      v = op(r16.x, r16.y);
      const float2 r32 = pair32(v);
      v = op(r32.x, r32.y);
    }
  }
  return v;
}

// first arg-max over one axis (lowest index wins ties); one-time use, shuffles are fine
template <int KP, bool INNER>
__device__ __forceinline__ void allargmax(float& v, int& a) {
#pragma unroll
  for (int o = INNER ? 1 : KP; o < (INNER ? KP : KP * KP); o <<= 1) {
    const float ov = __shfl_xor(v, o);
    const int oa = __shfl_xor(a, o);
    if (ov > v || (ov == v && oa < a)) { v = ov; a = oa; }
  }
}

// ---------------------------------------------------------------- table staging
// Chunk c of the wave's SPW sequences (b0 .. b0 + SPW - 1, clamped to B - 1)
// into one ring slot: [SPW][HC][K][K] log_A then [SPW][HC][K] em.  Steps past
// T read clamped (valid, unused) addresses.
template <int K, bool W16>
__device__ __forceinline__ void stage_chunk(const float* __restrict__ A, const float* __restrict__ E, int64_t b0,
                                            int64_t B, int T, int c, float* slot, int lane) {
  using Gm = Geo<K, W16>;
  using Rg = Ring<K, W16>;
  constexpr int U = Rg::U;
#pragma unroll
  for (int q = 0; q < Rg::NI; ++q) {
    const int f = (q * 64 + lane) * U;
    auto a_src = [&]() {
      const int sq = f / Gm::AS, off = f - sq * Gm::AS;
      const int64_t b = b0 + sq < B ? b0 + sq : B - 1;
      int64_t o = (int64_t)c * Gm::AS + off;
      const int64_t lim = (int64_t)T * K * K - U;
      o = o < lim ? o : lim;
      return A + b * (int64_t)T * K * K + o;
    };
    auto e_src = [&]() {
      const int fe = f - Gm::SPW * Gm::AS;
      const int sq = fe / Gm::ES, off = fe - sq * Gm::ES;
      const int64_t b = b0 + sq < B ? b0 + sq : B - 1;
      int64_t o = (int64_t)c * Gm::ES + off;
      const int64_t lim = (int64_t)T * K - U;
      o = o < lim ? o : lim;
      return E + b * (int64_t)T * K + o;
    };
    const float* src;
    if ((q + 1) * 64 * U <= Gm::SPW * Gm::AS) src = a_src();        // whole instruction in log_A
    else if (q * 64 * U >= Gm::SPW * Gm::AS) src = e_src();         // whole instruction in em
    else src = f < Gm::SPW * Gm::AS ? a_src() : e_src();
    auto* dst = (__attribute__((address_space(3))) void*)(slot + q * 64 * U);
    if constexpr (W16) __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds(src, dst, 4, 0, 0);
  }
}

// per-lane LDS offsets of the (i, j) entry / emission j for both step parities
template <int K, bool W16, class Gm = Geo<K, W16>>
struct LaneMap {
  int a_off[2], e_off[2];
  bool a_ok[2], e_ok[2];
  __device__ LaneMap(int grp, int g) {
    constexpr int KP = Gm::KP;
#pragma unroll
    for (int p = 0; p < 2; ++p) {  // p = 0: even t (outer), 1: odd t (inner)
      const int i = p == 0 ? g / KP : g % KP;
      const int j = p == 0 ? g % KP : g / KP;
      a_ok[p] = i < K && j < K;
      e_ok[p] = j < K;
      a_off[p] = grp * Gm::AS + (a_ok[p] ? i * K + j : 0);
      e_off[p] = Gm::SPW * Gm::AS + grp * Gm::ES + (e_ok[p] ? j : 0);
    }
  }
};

// --------------------------------------------------------------------- Viterbi
// bp map of one step for one sequence: byte j = lowest i with (v == max) at (i, j).
template <int KP>
__device__ __forceinline__ uint64_t transpose_bits(uint64_t x) {  // bit r*KP + c <-> c*KP + r
  if constexpr (KP == 8) {
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull; x ^= t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull; x ^= t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull; x ^= t ^ (t << 28);
  } else if constexpr (KP == 4) {
    uint64_t t;
    t = (x ^ (x >> 3)) & 0x0A0Aull; x ^= t ^ (t << 3);
    t = (x ^ (x >> 6)) & 0x00CCull; x ^= t ^ (t << 6);
  } else {
    const uint64_t t = (x ^ (x >> 1)) & 0x2ull;
    x ^= t ^ (t << 1);
  }
  return x;
}

template <int K>
__device__ __forceinline__ uint2 bp_map(uint32_t mlo, uint32_t mhi, int q, bool odd) {
  using Gm = Geo<K, false>;
  constexpr int KP = Gm::KP, G = Gm::G;
  uint64_t f = ((uint64_t)mhi << 32) | mlo;
  if constexpr (G < 64) f = (f >> (q * G)) & ((1ull << G) - 1);
  // odd t (inner map): bit g = j*KP + i, row j = the i's -> no transpose
  if (!odd) f = transpose_bits<KP>(f);
  uint32_t w[2] = {0u, 0u};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t row = (uint32_t)(f >> (j * KP)) & ((1u << KP) - 1);
    const uint32_t bj = (uint32_t)__builtin_ctz(row | (1u << KP)) & (KP - 1);
    w[j >> 2] |= bj << (8 * (j & 3));
  }
  return make_uint2(w[0], w[1]);
}

// lanes BASE .. BASE+7 of (lo, hi) = the 8 ballots.  One asm block: its
// s_nop sits after every ballot's v_cmp (they are its inputs), covering the
// "VALU writes SGPR -> v_writelane reads it" hazard once per 8 steps.
template <int BASE>
__device__ __forceinline__ void writelane8(uint32_t& lo, uint32_t& hi, const uint64_t* b) {
  asm("s_nop 4\n\t"
      "v_writelane_b32 %0, %2, %18\n\tv_writelane_b32 %1, %3, %18\n\t"
      "v_writelane_b32 %0, %4, %19\n\tv_writelane_b32 %1, %5, %19\n\t"
      "v_writelane_b32 %0, %6, %20\n\tv_writelane_b32 %1, %7, %20\n\t"
      "v_writelane_b32 %0, %8, %21\n\tv_writelane_b32 %1, %9, %21\n\t"
      "v_writelane_b32 %0, %10, %22\n\tv_writelane_b32 %1, %11, %22\n\t"
      "v_writelane_b32 %0, %12, %23\n\tv_writelane_b32 %1, %13, %23\n\t"
      "v_writelane_b32 %0, %14, %24\n\tv_writelane_b32 %1, %15, %24\n\t"
      "v_writelane_b32 %0, %16, %25\n\tv_writelane_b32 %1, %17, %25"
      : "+v"(lo), "+v"(hi)
      : "s"((uint32_t)b[0]), "s"((uint32_t)(b[0] >> 32)), "s"((uint32_t)b[1]), "s"((uint32_t)(b[1] >> 32)),
        "s"((uint32_t)b[2]), "s"((uint32_t)(b[2] >> 32)), "s"((uint32_t)b[3]), "s"((uint32_t)(b[3] >> 32)),
        "s"((uint32_t)b[4]), "s"((uint32_t)(b[4] >> 32)), "s"((uint32_t)b[5]), "s"((uint32_t)(b[5] >> 32)),
        "s"((uint32_t)b[6]), "s"((uint32_t)(b[6] >> 32)), "s"((uint32_t)b[7]), "s"((uint32_t)(b[7] >> 32)),
        "i"(BASE), "i"(BASE + 1), "i"(BASE + 2), "i"(BASE + 3), "i"(BASE + 4), "i"(BASE + 5), "i"(BASE + 6),
        "i"(BASE + 7));

}

__device__ __forceinline__ uint32_t perm_bytes(uint2 m, uint32_t sel) {
  return __builtin_amdgcn_perm(m.y, m.x, sel);
}

}  // namespace vqhmm
