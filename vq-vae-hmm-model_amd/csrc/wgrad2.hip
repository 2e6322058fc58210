// Weight/bias gradient of the small-channel convolutions (N, C <= 64), the
// split-K GEMM dW[n][c][tap] = sum_r dY[r][n] * X[r + tap - 1][c] over all PCL
// rows (pad rows of dY are zero, so the sum needs no masks).
//
//  * Persistent workgroups, one contiguous row chunk each; the chunk is walked
//    in 64-row stages whose dY / X tiles are prefetched into registers (float4
//    where the channel count allows, clamped + selected, no branches) while the
//    MFMAs of the previous stage run.
//  * The 4 waves split the work WN x WC x WR = 4 ways over (n-blocks, c-blocks,
//    16-row slices of each stage): large outputs (64x64x3) split the output
//    blocks, tiny ones (3x32, 10x64) also split the rows and add the partials
//    of the WR row-waves in a fixed order at the end.
//  * Per workgroup the partial dW (and dbias) goes to a slab; reduce_slabs sums
//    the slabs in a fixed order (deterministic, no atomics).
#include <stdlib.h>

#include <utility>

#include "kernels.h"

namespace vqhmm {

namespace {
constexpr int RT = 64;     // rows per stage (the output-heavy jobs)
constexpr int RT_S = 96;   // rows per stage of the small jobs (< 4096 outputs: MFMA work per 64-row stage is
                           // a few dozen MFMAs per wave, so the stage's loads, stores and two barriers set
                           // the time; 1.5x the rows, 2/3 of the stages: 128 or more push the group kernel
                           // past 256 registers, i.e. to one wave per SIMD)
constexpr int RT_S4 = 128;  // ... for the 4-row-wave body (its 16-row slices must split evenly over 4 waves)
}

// LDS floats of one wgrad2 body: dY stage, X stage (two of each double-buffered), bias partials, row-wave
// exchange
template <int NPAD, int CPAD, int RTV = RT, bool DB = false>
constexpr int w2_lds_floats() { return (DB ? 2 : 1) * (RTV * (NPAD + 4) + (RTV + 2) * (CPAD + 4)) + 256 + 1536; }
constexpr int w2_max(int a, int b) { return a > b ? a : b; }
// the group launch's dynamic LDS: the largest body (64x64 at RT, 16x64 / 64x16 small jobs at RT_S)
template <bool DB>
constexpr int w2_lds_max() {
  return w2_max(w2_max(w2_lds_floats<64, 64, RT, DB>(), w2_lds_floats<16, 16, RT_S4, DB>()),
                w2_max(w2_lds_floats<16, 64, RT_S, DB>(), w2_lds_floats<64, 16, RT_S, DB>()));
}

// The composed decoder conv1's embedding-gradient share of one chunk (WgradArgs::cmpW; N = H <= 64 outputs o,
// C = K <= 8 inputs k): cmp_slab[chunk][k][h] = sum_{o, tap} dWc[o][k][tap] W[o][h][tap] from the chunk's dWc
// in LDS (cbuf[(o * 3 + tap) * 8 + k], zero for k >= K and o >= H, so the loop below has no branch: the group
// kernel's code is large, and a branchy epilogue executed once per workgroup measured 13 us of instruction
// fetch); 4 thread groups split o (o = g, g + 4, ...), combined in a fixed order through part (4 * 8 * 64
// floats, the free stage buffer).  dE = sum over chunks (the backward tail).
__device__ __forceinline__ void wgrad_compose_de(const WgradArgs& a, int64_t chunk, const float* cbuf, float* part) {
  const int H = a.N, K = a.C, tid = threadIdx.x, h = tid & 63, g = tid >> 6;
  // all 48 weight loads in flight at once (clamped addresses), across the barrier that publishes cbuf
  float w[16][3];
  const int hc = min(h, H - 1);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int o = min(g + 4 * i, H - 1);
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) w[i][tap] = a.cmpW[((int64_t)o * H + hc) * 3 + tap];
  }
  __syncthreads();  // cbuf (this chunk's dWc) complete
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
      const float4* c4 = reinterpret_cast<const float4*>(cbuf + ((g + 4 * i) * 3 + tap) * 8);
      const float4 lo = c4[0], hi = c4[1];
      const float cv[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = fmaf(cv[k], w[i][tap], acc[k]);
    }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[(g * 8 + k) * 64 + h] = acc[k];
  __syncthreads();
  for (int i = tid; i < K * H; i += 256) {
    const int k = i / H, hh = i - k * H;
    const float v = ((part[k * 64 + hh] + part[(8 + k) * 64 + hh]) + part[(16 + k) * 64 + hh]) + part[(24 + k) * 64 + hh];
    a.cmp_slab[chunk * K * H + i] = v;
  }
}

// One chunk (workgroup) of the split-K weight gradient; smem = w2_lds_floats<NPAD, CPAD>() floats.
// PK (k = 3, 3*C <= 16): the three taps share ONE 16-wide MFMA column block, column j = tap*C + c
// (a per-lane gather from the X stage), so a narrow-input layer (enc_conv1 C = 5, the composed
// decoder conv1 C = K = 3) issues a third of the MFMAs of the tap-major form.
// DB: the dY / X stages double-buffered in LDS: stage s + 1 is stored from its prefetch registers into the
// other buffer while stage s's MFMAs run, one barrier per stage (single-buffered: store, barrier, MFMAs,
// barrier)
template <int NBW, int CBW, int KS, int NPAD, int CPAD, int WR, bool PK = false, int RT = vqhmm::RT, bool DB = false>
__device__ __forceinline__ void wgrad2_body(const WgradArgs& a, int WN, int WC, int64_t chunk, float* smem) {
  static_assert(!PK || (KS == 3 && CBW == 1), "packed taps: k = 3, one column block");
  constexpr int KA = PK ? 1 : KS;  // accumulator tap blocks
  constexpr int LDA = NPAD + 4, LDB = CPAD + 4;  // 4*LD = 16 (mod 32): conflict-free b32 column reads
  constexpr int DY4 = RT * NPAD / 4;             // float4 slots of the dY stage
  constexpr int X4 = (RT + 2) * CPAD / 4;        // float4 slots of the X stage
  constexpr int PD = (DY4 + 255) / 256, PX = (X4 + 255) / 256;
  constexpr int STG = RT * LDA + (RT + 2) * LDB;  // one dY + X stage
  float* dys = smem;                             // [RT][LDA] (buffer 0)
  float* xs = dys + RT * LDA;                    // [RT + 2][LDB]
  float* bred = smem + (DB ? 2 : 1) * STG;       // [256]
  float* xbuf = bred + 256;                      // [1536] row-wave exchange (WR > 1 only with NBW = CBW = 1)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int wr = wave % WR, wc = (wave / WR) % WC, wn = wave / (WR * WC);
  const int64_t rbeg = chunk * a.rows_per_chunk;
  const int64_t rend = min(a.R, rbeg + a.rows_per_chunk);

  // Raw float4 loads from clamped addresses (row strides ld4(N), ld4(C); pad
  // channels are zero in memory).  No select next to a load, so the prefetch
  // stays in flight across the MFMAs; rows outside the chunk / channels past
  // the row are zeroed when the registers are written to LDS.
  const int ldn = a.ld_dy ? a.ld_dy : ld4(a.N), ldc = ld4(a.C);
  auto load_dy = [&](int64_t r0, float4* p) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int s = tid + k * 256;
      const int row = s / (NPAD / 4), c = (s - row * (NPAD / 4)) * 4;
      int64_t r = r0 + row;
      r = r < rend ? r : rend - 1;
      p[k] = *reinterpret_cast<const float4*>(a.dy + r * ldn + min(c, ldn - 4));
    }
  };
  auto mask_dy = [&](int64_t r0, int k, float4 v) __attribute__((always_inline)) {
    const int s = tid + k * 256;
    const int row = s / (NPAD / 4), c = (s - row * (NPAD / 4)) * 4;
    return (r0 + row < rend && c < ldn) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto load_x = [&](int64_t r0, float4* p) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int s = tid + k * 256;
      const int row = s / (CPAD / 4), c = (s - row * (CPAD / 4)) * 4;
      int64_t r = r0 - 1 + row;
      r = r < 0 ? 0 : (r >= a.R ? a.R - 1 : r);
      p[k] = *reinterpret_cast<const float4*>(a.x + r * ldc + min(c, ldc - 4));
    }
  };
  auto mask_x = [&](int64_t r0, int k, float4 v) __attribute__((always_inline)) {
    const int s = tid + k * 256;
    const int row = s / (CPAD / 4), c = (s - row * (CPAD / 4)) * 4;
    const int64_t r = r0 - 1 + row;
    return (r >= 0 && r < a.R && c < ldc) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  };

  // packed taps: this lane's column j = l16 -> (tap, c)
  const int ptap = PK ? l16 / a.C : 0, pcc = PK ? l16 - (l16 / a.C) * a.C : 0;
  const bool pvalid = PK && l16 < 3 * a.C;
  f32x4 acc[KA][NBW][CBW];
#pragma unroll
  for (int tp = 0; tp < KA; ++tp)
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
      for (int j = 0; j < CBW; ++j) acc[tp][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  constexpr int bstep = 256 / NPAD;
  static_assert(RT % bstep == 0, "bias rows per thread");
  const int bcol = tid % NPAD, brow0 = tid / NPAD;

  float4 pdy[PD], px[PX];
  load_dy(rbeg, pdy);
  load_x(rbeg, px);
  if (a.cmpW)  // the composed epilogue's dWc buffer: entries no MFMA lane writes (k >= K, o >= H) stay zero
    for (int i = tid; i < 1536; i += 256) xbuf[i] = 0.f;
  // a stage's dY / X rows from the prefetch registers into LDS buffer (db, xb)
  auto store_stage = [&](int64_t r0, float* db, float* xb) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int s = tid + k * 256;
      if (s < DY4) {
        const int row = s / (NPAD / 4), c = (s - row * (NPAD / 4)) * 4;
        *reinterpret_cast<float4*>(db + row * LDA + c) = mask_dy(r0, k, pdy[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int s = tid + k * 256;
      if (s < X4) {
        const int row = s / (CPAD / 4), c = (s - row * (CPAD / 4)) * 4;
        *reinterpret_cast<float4*>(xb + row * LDB + c) = mask_x(r0, k, px[k]);
      }
    }
  };
  // bias partials and this wave's MFMAs over a stored stage
  auto compute = [&](const float* dys, const float* xs) __attribute__((always_inline)) {
      if (a.bias_slab) {  // RT / bstep rows per thread for every thread (RT % bstep == 0): all reads in flight
        float bp[RT / bstep];
#pragma unroll
        for (int k = 0; k < RT / bstep; ++k) bp[k] = dys[(brow0 + k * bstep) * LDA + bcol];
#pragma unroll
        for (int k = 0; k < RT / bstep; ++k) bacc += bp[k];
      }
      // this wave's 16-row slices of the stage, as 4 * (4 / WR) MFMA steps (one row per lane group
      // each): the operands of step s + 1 are read from LDS while the MFMAs of step s run (two
      // register sets, sched_barrier keeps the reads ahead); each accumulator's chain is unchanged
      static_assert((RT / 16) % WR == 0 && RT % 16 == 0, "a stage's 16-row slices split evenly over the row-waves");
      constexpr int NST = 4 * ((RT / 16) / WR);
      float av[2][NBW], bv[2][KA][CBW];
      auto load = [&](int st, float (&a_)[NBW], float (&b_)[KA][CBW]) __attribute__((always_inline)) {
        const int sl = wr + (st >> 2) * WR, e = st & 3;
        const int rr = sl * 16 + 4 * lg4 + e;
#pragma unroll
        for (int i = 0; i < NBW; ++i) a_[i] = dys[rr * LDA + (wn + i * WN) * 16 + l16];
        if constexpr (PK) {
          const float xv = xs[(rr + ptap) * LDB + pcc];
          b_[0][0] = pvalid ? xv : 0.f;
        } else {
#pragma unroll
          for (int tp = 0; tp < KS; ++tp) {
            const int xrow = rr + (KS == 3 ? tp : 1);
#pragma unroll
            for (int j = 0; j < CBW; ++j) b_[tp][j] = xs[xrow * LDB + (wc + j * WC) * 16 + l16];
          }
        }
      };
      load(0, av[0], bv[0]);
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        const int cb = st & 1;
        if (st + 1 < NST) load(st + 1, av[cb ^ 1], bv[cb ^ 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tp = 0; tp < KA; ++tp)
#pragma unroll
          for (int j = 0; j < CBW; ++j)
#pragma unroll
            for (int i = 0; i < NBW; ++i) acc[tp][i][j] = mfma16x16x4(av[cb][i], bv[cb][tp][j], acc[tp][i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
  };
  if constexpr (!DB) {
    for (int64_t r0 = rbeg; r0 < rend; r0 += RT) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < PD; ++k) {
        const int s = tid + k * 256;
        if (s < DY4) {
          const int row = s / (NPAD / 4), c = (s - row * (NPAD / 4)) * 4;
          *reinterpret_cast<float4*>(dys + row * LDA + c) = mask_dy(r0, k, pdy[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        const int s = tid + k * 256;
        if (s < X4) {
          const int row = s / (CPAD / 4), c = (s - row * (CPAD / 4)) * 4;
          *reinterpret_cast<float4*>(xs + row * LDB + c) = mask_x(r0, k, px[k]);
        }
      }
      __syncthreads();
      if (r0 + RT < rend) {
        load_dy(r0 + RT, pdy);
        load_x(r0 + RT, px);
      }
      compute(dys, xs);
    }
  } else {
    store_stage(rbeg, dys, xs);
    if (rbeg + RT < rend) {
      load_dy(rbeg + RT, pdy);
      load_x(rbeg + RT, px);
    }
    __syncthreads();
    int sb = 0;
    for (int64_t r0 = rbeg; r0 < rend; r0 += RT, sb ^= 1) {
      float* const cd = smem + sb * STG;   // this stage
      float* const nd = smem + (sb ^ 1) * STG;  // the next one, stored while this one's MFMAs run
      compute(cd, cd + RT * LDA);
      if (r0 + RT < rend) {
        store_stage(r0 + RT, nd, nd + RT * LDA);
        if (r0 + 2 * RT < rend) {
          load_dy(r0 + 2 * RT, pdy);
          load_x(r0 + 2 * RT, px);
        }
      }
      __syncthreads();  // the next stage stored; this stage's buffer free for the one after
    }
  }
  // ---- combine the WR row-waves (fixed order), then write the partial
  float* xch = xbuf;
  for (int w = 1; w < WR; ++w) {
    __syncthreads();
    if (wr == w) {
#pragma unroll
      for (int tp = 0; tp < KA; ++tp)
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
          for (int j = 0; j < CBW; ++j)
#pragma unroll
            for (int v = 0; v < 4; ++v)
              xch[(wave / WR) * (KA * NBW * CBW * 4 * 64) + (((tp * NBW + i) * CBW + j) * 4 + v) * 64 + lane] =
                  acc[tp][i][j][v];
    }
    __syncthreads();
    if (wr == 0) {
#pragma unroll
      for (int tp = 0; tp < KA; ++tp)
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
          for (int j = 0; j < CBW; ++j)
#pragma unroll
            for (int v = 0; v < 4; ++v)
              acc[tp][i][j][v] +=
                  xch[(wave / WR) * (KA * NBW * CBW * 4 * 64) + (((tp * NBW + i) * CBW + j) * 4 + v) * 64 + lane];
    }
  }
  if (wr == 0) {
    float* out = a.slab + chunk * (int64_t)a.N * a.C * KS;
#pragma unroll
    for (int tp = 0; tp < KA; ++tp)
#pragma unroll
      for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int j = 0; j < CBW; ++j)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int n = (wn + i * WN) * 16 + 4 * lg4 + v;
            const int c = (wc + j * WC) * 16 + l16;
            if constexpr (PK) {
              if (n < a.N && pvalid) {
                out[((int64_t)n * a.C + pcc) * KS + ptap] = acc[tp][i][j][v];
                if (a.cmpW) xbuf[(n * 3 + ptap) * 8 + pcc] = acc[tp][i][j][v];
              }
            } else {
              if (n < a.N && c < a.C) {
                out[((int64_t)n * a.C + c) * KS + tp] = acc[tp][i][j][v];
                if (a.cmpW) xbuf[(n * 3 + tp) * 8 + c] = acc[tp][i][j][v];
              }
            }
          }
  }
  if (a.cmpW) wgrad_compose_de(a, chunk, xbuf, smem);  // the composed decoder conv1: this chunk's dE share
  if (a.bias_slab) {
    __syncthreads();
    bred[tid] = bacc;
    __syncthreads();
    if (tid < NPAD && tid < a.N) {
      float s = 0.f;
      for (int k = 0; k < bstep; ++k) s += bred[k * NPAD + tid];
      a.bias_slab[chunk * a.N + tid] = s;
    }
  }
}

template <int NBW, int CBW, int KS, int NPAD, int CPAD, int WR>
__global__ __launch_bounds__(256) void wgrad2_kernel(WgradArgs a, int WN, int WC) {
  extern __shared__ float4 smem4[];
  wgrad2_body<NBW, CBW, KS, NPAD, CPAD, WR>(a, WN, WC, blockIdx.x, reinterpret_cast<float*>(smem4));
}

// ---- all of a step's weight gradients in ONE launch (WgradGroup): workgroup b runs chunk
// b - blk0[j] of job j.  Each job is one of the launch shapes below (variant id = its row in
// w2_variant, +10 for k = 3), so every body keeps its own register/LDS layout; big jobs come
// first so their workgroups start first and the small ones fill the tail.
#define VQHMM_W2_VARIANTS(KSV, O)                                                       \
  case O + 0: wgrad2_body<4, 1, KSV, 64, 64, 1, false, RT, DB>(a, WN, WC, ch, sm); break;    \
  case O + 1: wgrad2_body<2, 1, KSV, 32, 64, 1, false, RT, DB>(a, WN, WC, ch, sm); break;    \
  case O + 2: wgrad2_body<1, 2, KSV, 64, 32, 1, false, RT, DB>(a, WN, WC, ch, sm); break;    \
  case O + 3: wgrad2_body<1, 1, KSV, 16, 64, 1, false, RT_S, DB>(a, WN, WC, ch, sm); break;  \
  case O + 4: wgrad2_body<1, 1, KSV, 64, 16, 1, false, RT_S, DB>(a, WN, WC, ch, sm); break;  \
  case O + 5: wgrad2_body<1, 1, KSV, 16, 32, 2, false, RT_S, DB>(a, WN, WC, ch, sm); break;  \
  case O + 6: wgrad2_body<1, 1, KSV, 32, 16, 2, false, RT_S, DB>(a, WN, WC, ch, sm); break;  \
  case O + 7: wgrad2_body<1, 1, KSV, 32, 32, 1, false, RT_S, DB>(a, WN, WC, ch, sm); break;  \
  case O + 8: wgrad2_body<1, 1, KSV, 16, 16, 4, false, RT_S4, DB>(a, WN, WC, ch, sm); break;

template <bool DB>
__global__ __launch_bounds__(256, 3) void wgrad2_group_kernel(WgradGroup g) {
  extern __shared__ float4 smem4[];
  float* sm = reinterpret_cast<float*>(smem4);  // w2_lds_max<DB>() floats
  if (g.step_inc && blockIdx.x == 0 && threadIdx.x == 0) *g.step_inc = (*g.step_inc & 0xffffffffll) + 1;
  int j = 0;
  while (j + 1 < g.njobs && (int64_t)blockIdx.x >= g.blk0[j + 1]) ++j;
  const WgradArgs& a = g.job[j];
  const int WN = g.wn[j], WC = g.wc[j];
  const int64_t ch = (int64_t)blockIdx.x - g.blk0[j];
  switch (g.variant[j]) {
    VQHMM_W2_VARIANTS(1, 0)
    VQHMM_W2_VARIANTS(3, 10)
    case 20: wgrad2_body<1, 1, 3, 64, 16, 1, true, RT_S, DB>(a, WN, WC, ch, sm); break;
    default: break;
  }
}
#undef VQHMM_W2_VARIANTS

// A/B switch: VQHMM_WGRAD_PACK=0 keeps the tap-major form for narrow inputs (read once)
static bool packed_taps() {
  static const bool v = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_PACK");
    return !(e && e[0] == '0');
  }();
  return v;
}

// launch shape of a job: variant id (see above) and its wave split (WN, WC); -1 if none
static int w2_variant(int N, int C, int ks, int* WN, int* WC) {
  const int nbn = (int)cdiv(N, 16), nbc = (int)cdiv(C, 16);
  int v;
  if (nbn == 4 && nbc == 4) { v = 0; *WN = 1; *WC = 4; }
  else if (nbn == 2 && nbc == 4) { v = 1; *WN = 1; *WC = 4; }
  else if (nbn == 4 && nbc == 2) { v = 2; *WN = 4; *WC = 1; }
  else if (nbn == 1 && nbc == 4) { v = 3; *WN = 1; *WC = 4; }
  else if (nbn == 4 && nbc == 1) { v = 4; *WN = 4; *WC = 1; }
  else if (nbn == 1 && nbc == 2) { v = 5; *WN = 1; *WC = 2; }
  else if (nbn == 2 && nbc == 1) { v = 6; *WN = 2; *WC = 1; }
  else if (nbn == 2 && nbc == 2) { v = 7; *WN = 2; *WC = 2; }
  else if (nbn == 1 && nbc == 1) { v = 8; *WN = 1; *WC = 1; }
  else if (nbn <= 4 && nbc <= 4) { v = 0; *WN = 1; *WC = 4; }
  else return -1;
  if (ks == 3 && nbn == 4 && 3 * C <= 16 && packed_taps()) return 20;  // taps packed into one block
  return v + (ks == 3 ? 10 : 0);
}

// rows per stage of a job in the grouped launch (variants 0..2 and 10..12 are the output-heavy bodies)
static int w2_group_rt(int variant) {
  const int v = variant % 10;
  return (variant < 20 && v <= 2) ? RT : (variant < 20 && v == 8) ? RT_S4 : RT_S;
}

// a grouped job's rows per chunk: `rows` rounded up to its stage size
int64_t wgrad2_group_rows(int64_t rows, int N, int C, int ks) {
  int wn, wc;
  const int v = w2_variant(N, C, ks, &wn, &wc);
  const int rt = v < 0 ? RT : w2_group_rt(v);
  return cdiv(rows, rt) * rt;
}

bool wgrad2_group_supported(const WgradArgs& a) {
  int wn, wc;
  const int v = w2_variant(a.N, a.C, a.ks, &wn, &wc);
  if (a.x_cf || a.N > 64 || a.C > 64 || (a.ks != 1 && a.ks != 3) || v < 0) return false;
  // the composed epilogue: dWc fits the row-wave buffer (1536 floats), one row-wave, K <= 8 accumulators
  if (a.cmpW) return a.ks == 3 && a.C <= 8 && a.N * a.C * 3 <= 1536 && (v == 20 || (v % 10 != 5 && v % 10 != 6 && v % 10 != 8));
  return true;
}

int launch_wgrad2_group(const WgradArgs* jobs, int n, hipStream_t s, int64_t* step_inc) {
  if (n < 1 || n > MAX_WJOBS) return VQHMM_EINVAL;
  WgradGroup g{};
  g.step_inc = step_inc;
  // biggest outputs first (their chunks run longest)
  int ord[MAX_WJOBS];
  for (int i = 0; i < n; ++i) ord[i] = i;
  for (int i = 1; i < n; ++i)
    for (int k = i; k > 0; --k) {
      const WgradArgs &x = jobs[ord[k]], &y = jobs[ord[k - 1]];
      if ((int64_t)x.N * x.C * x.ks > (int64_t)y.N * y.C * y.ks) std::swap(ord[k], ord[k - 1]);
    }
  g.njobs = n;
  g.blk0[0] = 0;
  for (int i = 0; i < n; ++i) {
    const WgradArgs& a = jobs[ord[i]];
    if (!wgrad2_group_supported(a)) return VQHMM_EINVAL;
    g.job[i] = a;
    g.variant[i] = w2_variant(a.N, a.C, a.ks, &g.wn[i], &g.wc[i]);
    if (a.rows_per_chunk % w2_group_rt(g.variant[i])) return VQHMM_EINVAL;
    g.blk0[i + 1] = g.blk0[i] + cdiv(a.R, a.rows_per_chunk);
  }
  if (g.blk0[n] == 0) return VQHMM_OK;
  // A/B (profiling build): VQHMM_WGRAD_DB=1 double-buffers the dY / X stages (one barrier per stage)
  static const bool db = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_DB");
    return e && e[0] == '1';
  }();
  if (db) wgrad2_group_kernel<true><<<(unsigned)g.blk0[n], 256, w2_lds_max<true>() * sizeof(float), s>>>(g);
  else wgrad2_group_kernel<false><<<(unsigned)g.blk0[n], 256, w2_lds_max<false>() * sizeof(float), s>>>(g);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

bool wgrad2_supported(const WgradArgs& a) { return !a.x_cf && a.N <= 64 && a.C <= 64; }

// chunks per launch for big outputs (tuning override VQHMM_WGRAD_BIG_CHUNKS, read once).  192: with
// the grouped launch the small jobs fill the CUs, and fewer, longer chunks mean less slab traffic and a
// shorter tail (cfg2 step 128 / 192 / 256 / 512 chunks: 0.4735 / 0.4728 / 0.4817 / 0.485 ms)
static int64_t big_chunks() {
  static const int64_t n = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_BIG_CHUNKS");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v >= 64 && v <= 4096 ? v : 192);
  }();
  return n;
}

// chunks for every output size (experiment override VQHMM_WGRAD_CHUNKS, read once; 0 = default)
static int64_t all_chunks() {
  static const int64_t n = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_CHUNKS");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v >= 64 && v <= 65536 ? v : 0);
  }();
  return n;
}

// chunks for small outputs (N * C * ks < 4096; override VQHMM_WGRAD_SMALL_CHUNKS, read once)
static int64_t small_chunks() {
  static const int64_t n = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_SMALL_CHUNKS");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v >= 64 && v <= 4096 ? v : 512);
  }();
  return n;
}

int64_t wgrad2_rows(int64_t R, int N, int C, int ks) {
  int64_t chunks = ((int64_t)N * C * ks >= 4096) ? big_chunks() : small_chunks();
  if (all_chunks()) chunks = all_chunks();
  int64_t rows = cdiv(R, chunks);
  return cdiv(rows, RT) * RT;
}

template <int NBW, int CBW, int KS, int NPAD, int CPAD, int WR>
static int launch_w2(const WgradArgs& a, int WN, int WC, hipStream_t s) {
  const int64_t nchunks = cdiv(a.R, a.rows_per_chunk);
  if (WR > 1 && (NBW * CBW != 1 || KS * 4 * 64 * (4 / WR) > 1536)) return VQHMM_EUNSUPPORTED;
  if (WN * WC * WR != 4) return VQHMM_EINVAL;
  WgradArgs ap = a;
  wgrad2_kernel<NBW, CBW, KS, NPAD, CPAD, WR>
      <<<(unsigned)nchunks, 256, w2_lds_floats<NPAD, CPAD>() * sizeof(float), s>>>(ap, WN, WC);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

template <int KS>
static int launch_w2_ks(const WgradArgs& a, hipStream_t s) {
  const int nbn = (int)cdiv(a.N, 16), nbc = (int)cdiv(a.C, 16);
  // choose the wave split: prefer output blocks, then rows
  if (nbn == 4 && nbc == 4) return launch_w2<4, 1, KS, 64, 64, 1>(a, 1, 4, s);
  if (nbn == 2 && nbc == 4) return launch_w2<2, 1, KS, 32, 64, 1>(a, 1, 4, s);
  if (nbn == 4 && nbc == 2) return launch_w2<1, 2, KS, 64, 32, 1>(a, 4, 1, s);
  if (nbn == 1 && nbc == 4) return launch_w2<1, 1, KS, 16, 64, 1>(a, 1, 4, s);
  if (nbn == 4 && nbc == 1) return launch_w2<1, 1, KS, 64, 16, 1>(a, 4, 1, s);
  if (nbn == 1 && nbc == 2) return launch_w2<1, 1, KS, 16, 32, 2>(a, 1, 2, s);
  if (nbn == 2 && nbc == 1) return launch_w2<1, 1, KS, 32, 16, 2>(a, 2, 1, s);
  if (nbn == 2 && nbc == 2) return launch_w2<1, 1, KS, 32, 32, 1>(a, 2, 2, s);
  if (nbn == 1 && nbc == 1) return launch_w2<1, 1, KS, 16, 16, 4>(a, 1, 1, s);
  if (nbn <= 4 && nbc <= 4) return launch_w2<4, 1, KS, 64, 64, 1>(a, 1, 4, s);
  return VQHMM_EUNSUPPORTED;
}

int launch_wgrad2(const WgradArgs& a, hipStream_t s) {
  if (a.R == 0) return VQHMM_OK;
  return a.ks == 3 ? launch_w2_ks<3>(a, s) : launch_w2_ks<1>(a, s);
}

}  // namespace vqhmm
