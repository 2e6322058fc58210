// Strip kernels: several convolution layers of the training step in ONE launch, the activations
// between the layers kept in LDS (VQ_VAE_HMM_fixed.py:38-41 Encoder.forward, :80-90 Decoder.forward).
//
// A strip is a window of ST_WIN = 128 consecutive PCL rows whose middle ST_OWN = 124 rows it owns
// (owned rows tile [0, R) without overlap).  Wave w of the 8-wave workgroup owns the window's
// 16-row block w through the whole chain
//   x -> enc_conv1 -> enc_conv2 (+ to_logits, softmax) -> composed dec_conv1 -> dec_conv2 (+ to_params).
// The narrow front convs (enc_conv1 on x, dec_conv1 on q: packed taps, 16 MFMAs a block) are computed
// by the wave itself for the 18 rows its 64-wide conv reads (two overlapping MFMA blocks) into its own
// LDS slot, so only q (and the next strip's x) cross waves: two workgroup barriers per strip.  The
// window's outer rows are inexact after the k = 3 layers (x is loaded with a 2-row halo), so a strip
// stores rows >= ST_HALO = 2 from its edges only: 3% recomputed rows replace four launches' fixed
// costs (weight staging, the first tile's latency, the tail) with one — what bounds the step at the
// strong-scaling shard sizes (B = 128 per GPU).
//
// Every row goes through the pair launches' MFMA sequences and epilogue arithmetic (conv2_dev.h), so
// the stored activations are the same bits as the conv2f path (tests: strip = pair launches).
#include "vqhmm.h"

#include <stddef.h>
#include <stdlib.h>

#include "prof.h"
#include "strip_dev.h"

namespace vqhmm {

struct StripFwdArgs {
  int64_t R;
  int T, D, H2, K, P;  // P = 2D (to_params outputs)
  const float* xp;     // PCL x (R, ld4(D))
  const float *img_e1, *img_d1;  // packed-front images [3][64][24] (the prologue's)
  const float *img_e2, *img_d2;  // enc_conv2 [3][16 NB2][72] / dec_conv2 [3][64][72] images
  const float *b_e1, *b_e2, *b_d1, *b_d2;
  const float *tWl, *tbl;        // to_logits (K, H2), (K)
  const float *tWp, *tbp;        // to_params (P, 64), (P)
  float *h1e, *h2e, *logits, *q, *g1, *g2, *par;
  int64_t nstrip;
  int dbg;  // profiling experiments (VQHMM_STRIP_DBG, read once; results then invalid): 1 = no global stores
};

namespace {

template <int NB2>
struct StripFwdLds {
  static constexpr int NW2 = 16 * NB2;
  float We2[3 * NW2 * ST_LDW];  // enc_conv2 image
  float Wd2[3 * 64 * ST_LDW];   // dec_conv2 image
  float Ee2[NW2 * 17 + 16];     // enc_conv2 bias | to_logits weight (16 x NW2) | bias
  float Ed2[64 * 17 + 16];      // dec_conv2 bias | to_params weight (16 x 64) | bias
  float Wf[2][3 * 64 * 8];      // enc_conv1 / dec_conv1 images, channels 0..7 ([tap][n][8])
  float bf[2][64];              // enc_conv1 / dec_conv1 bias (Wf | bf: the fused head's weights after startup)
  float Xx[ST_XR * ST_XLD];     // x rows s0 - 2 .. s0 + 129
  float Xq[ST_XR * ST_XLD];     // q rows s0 - 2 .. s0 + 129 (the 2 + 2 outer rows stay zero)
  float slot[8][18 * ST_LDW];   // per wave: the 64-wide conv's 18 input rows rb - 1 .. rb + 16
  unsigned long long hcnt[8];   // fused head: per-wave valid counts
};

// The fused ELBO head's LDS (strip_fwd_kernel with HTH > 0): per strip in the slots region (free after
// dec_conv2's loops), the Prior MLP weights in the constants' region (free once they are in registers).
template <int TH>
struct StripHeadW {
  static constexpr int LDW2 = TH + 4;
  float W2S[16 * LDW2];  // rows ij >= K^2 zero
  float W1S[TH * 8];     // W1' = [W1 | b1 | 0]
};
struct StripHeadLds {
  static constexpr int LDL = 20;  // lgS / dlgS row stride (16 ij + 4)
  float uS[ST_WIN * 8];           // u' = [u, 1 at column U, 0]
  float lgS[ST_WIN * LDL];        // transition logits of the window's rows
  float dlgS[ST_WIN * LDL];       // their gradients (zero for ij >= K^2, non-owned rows)
  float aS[ST_WIN * 4];           // A_i = sum_j q[j] log_A[i][j] per row
  float wS[ST_WIN];               // pair weight (t - 1, t) per row
  double red[8][4];
  float q0w[8][4];
};

// A packed-tap front's weights as c2_mfma_pk gathers them (k-column 4 lg4 + e, channel nb*16 + l16),
// from the compact [tap][n][8] LDS image into registers for the whole launch; columns past 3C are 0
__device__ __forceinline__ void pk_weights(const float* Wf, int C, int lg4, int l16, float (&w)[4][4]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = 4 * lg4 + e;
    const bool in = k < 3 * C;
    const int tap = in ? k / C : 0, c = in ? k - tap * C : 0;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const float v = Wf[(tap * 64 + nb * 16 + l16) * 8 + c];
      w[nb][e] = in ? v : 0.f;
    }
  }
}

// One packed-tap front MFMA block (c2_mfma_pk's sequence): 16 output rows whose k = 3 inputs are rows
// Xw[l16 + tap] (stride ST_XLD); k-columns past 3C are 0 x 0.
__device__ __forceinline__ void pk_block(const float (&w)[4][4], const float* Xw, int C, int lg4, int l16,
                                         f32x4 (&acc)[4]) {
  float b[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = 4 * lg4 + e;
    const bool in = k < 3 * C;
    const int tap = in ? k / C : 0, c = in ? k - tap * C : 0;
    const float v = Xw[(l16 + tap) * ST_XLD + c];
    b[e] = in ? v : 0.f;
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[nb] = mfma16x16x4(w[nb][e], b[e], acc[nb]);
  }
}

// conv2_epilogue's ACT = 1 arithmetic on a 64-wide block (bias, ReLU, pad rows 0): rows r0 + l16;
// rows l16 in [slo, shi) are stored to out (PCL, 64 channels); rows go to the LDS slot rows xs (every row,
// or only row `only` when only >= 0), row 0 also to the row xlo and row 15 to the row xhi (when given).
__device__ __forceinline__ void front_epi(f32x4 (&acc)[4], const f32x4 (&bias)[4], int64_t r0, int64_t R, int T,
                                          int lg4, int l16, int slo, int shi, float* out, float* xs,
                                          bool nostore, int only = -1, float* xlo = nullptr,
                                          float* xhi = nullptr) {
  const int64_t r = r0 + l16;
  const bool valid = row_valid(r, R, T);
  const bool st = l16 >= slo && l16 < shi && r < R && !nostore;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    f32x4 y;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float yy = relu_f(acc[nb][v] * 1.0f + bias[nb][v]);
      y[v] = valid ? yy : 0.f;
    }
    acc[nb] = y;
    if (st) *reinterpret_cast<f32x4*>(out + r * 64 + nb * 16 + 4 * lg4) = y;
    if (only < 0 || l16 == only) *reinterpret_cast<f32x4*>(xs + l16 * ST_LDW + nb * 16 + 4 * lg4) = y;
    if (xlo && l16 == 0) *reinterpret_cast<f32x4*>(xlo + nb * 16 + 4 * lg4) = y;
    if (xhi && l16 == 15) *reinterpret_cast<f32x4*>(xhi + nb * 16 + 4 * lg4) = y;
  }
}

// The lane's epilogue constants of a [bias | tail weight | tail bias] block, held in registers
template <int NB>
struct TailConsts {
  f32x4 bias[NB], tw[NB], tb;
  __device__ __forceinline__ void load(const float* Es, int lg4, int l16) {
    constexpr int NW = 16 * NB;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const float4 b4 = *reinterpret_cast<const float4*>(Es + nb * 16 + 4 * lg4);
      const float4 t4 = *reinterpret_cast<const float4*>(Es + NW + l16 * NW + nb * 16 + 4 * lg4);
      bias[nb] = f32x4{b4.x, b4.y, b4.z, b4.w};
      tw[nb] = f32x4{t4.x, t4.y, t4.z, t4.w};
    }
    const float4 t4 = *reinterpret_cast<const float4*>(Es + 17 * NW + 4 * lg4);
    tb = f32x4{t4.x, t4.y, t4.z, t4.w};
  }
};

// conv2_epilogue's ACT = 1 + one-block 1x1 tail (+ softmax) arithmetic: y (NW channels, stored to out
// with row stride ldn), z = tail(y) (stored to t_out, stride ldt), q = softmax(z) (SM: to q_out and the
// LDS rows xq); rows l16 in [slo, shi) are stored.
template <int NB, bool SM>
__device__ __forceinline__ void tail_epi(f32x4 (&acc)[NB], const TailConsts<NB>& k, int64_t r0, int64_t R, int T,
                                         int lg4, int l16, int slo, int shi, int N, float* out, int C2, float* t_out,
                                         float* q_out, float* xq, bool nostore) {
  const int64_t r = r0 + l16;
  const bool valid = row_valid(r, R, T);
  const bool st = l16 >= slo && l16 < shi && r < R && !nostore;
  const int ldn = ld4(N), ldt = ld4(C2);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    f32x4 y;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float yy = relu_f(acc[nb][v] * 1.0f + k.bias[nb][v]);
      y[v] = valid ? yy : 0.f;
    }
    acc[nb] = y;
    const int n0 = nb * 16 + 4 * lg4;
    if (st && n0 < ldn) *reinterpret_cast<f32x4*>(out + r * ldn + n0) = y;
  }
  f32x4 z = k.tb;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int v = 0; v < 4; ++v) z = mfma16x16x4(k.tw[nb][v], acc[nb][v], z);
  const int c0 = 4 * lg4;
#pragma unroll
  for (int v = 0; v < 4; ++v) z[v] = valid ? z[v] : 0.f;
  if (st && c0 < ldt) *reinterpret_cast<f32x4*>(t_out + r * ldt + c0) = z;
  if constexpr (SM) {
    float m = -__builtin_inff();
#pragma unroll
    for (int v = 0; v < 4; ++v)
      if (c0 + v < C2) m = fmaxf(m, z[v]);
    m = fmaxf(m, xor16(m));
    m = fmaxf(m, xor32(m));
    float e[4], s = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      e[v] = (c0 + v < C2) ? __expf(z[v] - m) : 0.f;
      s += e[v];
    }
    s += xor16(s);
    s += xor32(s);
    f32x4 qv;
#pragma unroll
    for (int v = 0; v < 4; ++v) qv[v] = valid ? e[v] / s : 0.f;
    if (st && c0 < ldt) *reinterpret_cast<f32x4*>(q_out + r * ldt + c0) = qv;
    if (c0 == 0) {  // K <= 4: channels 0..3 of the row; the fused head reads the logits from 4..7
      *reinterpret_cast<f32x4*>(xq + l16 * ST_XLD) = qv;
      *reinterpret_cast<f32x4*>(xq + l16 * ST_XLD + 4) = z;
    }
  }
}

// the source address of element i of a [bias (NW) | tail weight (16 x NW) | tail bias (16)] block, branch-free
// (selects only, so a caller's loads of several entries are all in flight before one wait: a branchy form's
// loads each ended in a vmcnt(0) at the branch join, ~10 serialized loads of staging); !ok -> the entry is 0
// and the returned address is the (valid) bias pointer
template <int NW>
__device__ __forceinline__ const float* es_src(const float* bias, int N, const float* tW, const float* tb, int C2, int i,
                                               bool& ok) {
  const bool in_b = i < NW, in_w = !in_b && i < 17 * NW;
  const int j = in_w ? i - NW : 0, c2w = j / NW, n = j - c2w * NW, c2b = (!in_b && !in_w) ? i - 17 * NW : 0;
  ok = in_b ? i < N : in_w ? (c2w < C2 && n < N) : c2b < C2;
  const float* p = in_b ? bias + i : in_w ? tW + ((int64_t)c2w * N + n) : tb + c2b;
  return ok ? p : bias;
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, dpp_u32<CTRL>(__builtin_bit_cast(uint32_t, v)));
}
// reductions over the 4 lanes of a head row (lane % 4 = source state), as head_coop.hip's row_* (KP = 4)
__device__ __forceinline__ float row4_sum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  return v;
}
__device__ __forceinline__ float row4_max(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  return v;
}
__device__ __forceinline__ float row4_reduce_scatter(const float (&c)[4], int i) {
  const bool hi2 = i & 2, hi1 = i & 1;
  float h2[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float send = hi2 ? c[k] : c[2 + k];
    h2[k] = (hi2 ? c[2 + k] : c[k]) + dppf<0x4E>(send);
  }
  const float send = hi1 ? h2[0] : h2[1];
  return (hi1 ? h2[1] : h2[0]) + dppf<0xB1>(send);
}
}  // namespace

// HTH > 0: the ELBO head (head_coop.hip's phases, VQ_VAE_HMM_fixed.py:59-71 Prior MLP, :106-137 loss) runs
// on each strip's owned rows after its decoder, on the activations still in LDS (q, logits) or just written
// (mu | logvar): K <= 4, U <= 4, TH = HTH in {64, 128}, D <= 8; h = the head launch's arguments, its slabs
// and loss partials indexed by workgroup (grid = the head's slab count).
template <int NB2, int PROF, int HTH>
__global__ __launch_bounds__(512) void strip_fwd_kernel(StripFwdArgs a, HeadArgs h) {
  using S = StripFwdLds<NB2>;
  constexpr int NW2 = S::NW2;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int64_t R = a.R;
  const int T = a.T, ldx = ld4(a.D);
  float* slot = sh.slot[wave];

  // x rows s0 - 2 .. s0 + 129 of a window: thread i < 2 ST_XR holds float4 i % 2 of row i / 2;
  // the load is unconditional (clamped), the mask applied when it is stored
  auto load_x = [&](int64_t s0) {
    const int row = tid >> 1, h = 4 * (tid & 1);
    int64_t r = s0 - 2 + row;
    r = r < 0 ? 0 : (r >= R ? R - 1 : r);
    return *reinterpret_cast<const float4*>(a.xp + r * ldx + (h < ldx ? h : 0));
  };
  auto store_x = [&](int64_t s0, float4 v) {
    if (tid < 2 * ST_XR) {
      const int row = tid >> 1, h = 4 * (tid & 1);
      const int64_t r = s0 - 2 + row;
      const bool ok = r >= 0 && r < R && h < ldx;
      *reinterpret_cast<float4*>(sh.Xx + row * ST_XLD + h) = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  // ---- fused head (HTH > 0): thread = (row prow, source state si) in the head phases
  constexpr int HKP = 4, HB = HTH > 0 ? HTH / 16 : 1, HLDW2 = HTH + 4, HNW = HTH > 0 ? 16 * HLDW2 + HTH * 8 : 1;
  constexpr int HNJ = (HNW + 511) / 512;
  const int prow = tid >> 2, si = tid & 3;
  float hwv[HNJ];  // the Prior MLP weights as StripHeadW lays them out (LDS after the first q exchange)
  if constexpr (HTH > 0) {
    const int KK = h.K * h.K;
#pragma unroll
    for (int j = 0; j < HNJ; ++j) {
      const int i = tid + 512 * j;
      float v = 0.f;
      if (i < 16 * HLDW2) {
        const int ij = i / HLDW2, hh = i - ij * HLDW2;
        v = (ij < KK && hh < HTH) ? h.W2[ij * HTH + hh] : 0.f;
      } else if (i < HNW) {
        const int k = i - 16 * HLDW2, hh = k >> 3, c = k & 7;
        v = c < h.U ? h.W1[hh * h.U + c] : (c == h.U ? h.b1[hh] : 0.f);
      }
      hwv[j] = v;
    }
    if (!h.norm && !h.cnt_in) {  // valid positions of the batch (mask.sum(), :120)
      unsigned long long c = 0;
      for (int64_t b = tid; b < h.B; b += 512) {
        const int64_t L = h.lengths[b];
        c += (unsigned long long)(L <= 0 ? 0 : (L < T ? L : T));
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
      if (lane == 0) sh.hcnt[wave] = c;
    }
  }
  stamp<PROF>(0);
  if constexpr (PROF > 0) { if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 13] = __builtin_amdgcn_s_memtime(); }
  // ---- once.  vmcnt retires in order, so: the front images (LDS DMA) first, then x and the epilogue
  // constants (registers), then the two 64-wide images (LDS DMA): waiting for x / the constants never
  // waits for the big images, which stay in flight through the first enc_conv1.
  // Wf[img][row][8] <- image row (tap, n) channels 0..7, by waves 0..3 only: those store x before the
  // first barrier, so their wait for x (younger) covers these
  for (int j = wave; wave < 4 && j < 12; j += 4) {
    const int g = j * 64 + lane, img = g / 384, i = g - img * 384, row = i >> 1, h = 4 * (i & 1);
    dma16((img ? a.img_d1 : a.img_e1) + row * ST_LDF + h, &sh.Wf[0][0] + j * 256);
  }
  int64_t s = blockIdx.x;
  float4 px = load_x(s * ST_OWN - ST_HALO);
  constexpr int NE = NW2 * 17 + 16, ND = 64 * 17 + 16, NC = NE + ND + 128;  // sh.Ee2 | sh.Ed2 | sh.bf
  constexpr int NCJ = (NC + 511) / 512;
  float cv[NCJ];
  bool cvok[NCJ];
#pragma unroll
  for (int j = 0; j < NCJ; ++j) {
    const int i = tid + 512 * j;
    bool oke, okd;
    const float* pe = es_src<NW2>(a.b_e2, a.H2, a.tWl, a.tbl, a.K, i < NE ? i : 0, oke);
    const float* pd = es_src<64>(a.b_d2, 64, a.tWp, a.tbp, a.P, (i >= NE && i < NE + ND) ? i - NE : 0, okd);
    const int ib = (i >= NE + ND && i < NC) ? i - NE - ND : 0;
    const bool inE = i < NE, inD = !inE && i < NE + ND, inB = !inE && !inD && i < NC;
    const bool ok = inE ? oke : inD ? okd : inB;
    const float* p = inE ? pe : inD ? pd : (ib < 64 ? a.b_e1 : a.b_d1) + (ib & 63);
    cv[j] = *(ok ? p : a.b_e1);  // every entry's load in flight; the mask after the loop
    cvok[j] = ok;
  }
#pragma unroll
  for (int j = 0; j < NCJ; ++j) cv[j] = cvok[j] ? cv[j] : 0.f;
  {
    constexpr int N1 = 3 * NW2 * ST_LDW / 4, N2 = 3 * 64 * ST_LDW / 4;  // float4s of each image
    constexpr int C1 = (N1 + 63) / 64, C2 = (N2 + 63) / 64;              // one wave instruction = 1 KB
    // a fixed count per wave (the last chunk copied again where a wave has fewer: the same bytes), so the
    // compiler counts these in vmcnt and its waits for x / the constants below leave them in flight
    constexpr int NJ = (C1 + C2 + 7) / 8;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int c = min(wave + 8 * jj, C1 + C2 - 1);
      const bool first = c < C1;
      const int cc = first ? c : c - C1;
      const int i = cc * 64 + lane;
      if (i < (first ? N1 : N2)) dma16((first ? a.img_e2 : a.img_d2) + 4 * i, (first ? sh.We2 : sh.Wd2) + cc * 256);
    }
  }
  static_assert(offsetof(S, Ed2) == offsetof(S, Ee2) + NE * 4, "constant blocks must be contiguous");
#pragma unroll
  for (int j = 0; j < NCJ; ++j) {
    const int i = tid + 512 * j;
    if (i < NE + ND) sh.Ee2[i] = cv[j];
    else if (i < NC) sh.bf[0][i - NE - ND] = cv[j];
  }
  if (tid < 4 * ST_XLD) sh.Xq[(tid < 2 * ST_XLD ? 0 : (ST_XR - 4) * ST_XLD) + tid] = 0.f;  // rows never written
  store_x(s * ST_OWN - ST_HALO, px);
  lds_barrier();  // LDS only: the big images stay in flight (the front images are older than x: landed)
  stamp<PROF>(1);
  float wE[4][4], wD[4][4];
  pk_weights(sh.Wf[0], a.D, lg4, l16, wE);
  pk_weights(sh.Wf[1], a.K, lg4, l16, wD);
  f32x4 bE[4], bD[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const float4 e4 = *reinterpret_cast<const float4*>(sh.bf[0] + nb * 16 + 4 * lg4);
    const float4 d4 = *reinterpret_cast<const float4*>(sh.bf[1] + nb * 16 + 4 * lg4);
    bE[nb] = f32x4{e4.x, e4.y, e4.z, e4.w};
    bD[nb] = f32x4{d4.x, d4.y, d4.z, d4.w};
  }
  // the tail epilogues' constants: registers, or (with the fused head, whose phases need the registers)
  // re-read from LDS for every tile
  TailConsts<NB2> kE;
  TailConsts<4> kD;
  if constexpr (HTH == 0) {
    kE.load(sh.Ee2, lg4, l16);
    kD.load(sh.Ed2, lg4, l16);
  }
  static_assert(HTH == 0 || (offsetof(S, Xx) == offsetof(S, bf) + 2 * 64 * 4 &&
                             sizeof(StripHeadW<HTH>) <= offsetof(S, Xx) - offsetof(S, Wf) &&
                             sizeof(StripHeadLds) <= sizeof(float) * 8 * 18 * ST_LDW),
                "the head's LDS fits the regions it reuses");
  float lp_i = 0.f, inv_n = 1.f, cpri = 0.f, cent = 0.f;
  const bool hgrad = h.need_grad != 0;
  if constexpr (HTH > 0) {
    unsigned long long cnt;
    if (h.norm) cnt = (unsigned long long)h.norm[0];
    else if (h.cnt_in) cnt = (unsigned long long)*h.cnt_in;
    else cnt = ((((((sh.hcnt[0] + sh.hcnt[1]) + sh.hcnt[2]) + sh.hcnt[3]) + sh.hcnt[4]) + sh.hcnt[5]) + sh.hcnt[6]) + sh.hcnt[7];
    inv_n = 1.0f / fmaxf((float)(cnt * (unsigned long long)h.D), 1.0f);
    const float Bn = loss_norm_batch(h.norm, h.B);
    cpri = -h.beta / Bn;
    cent = h.beta / Bn;
    float m = -__builtin_inff();
    for (int k = 0; k < h.K; ++k) m = fmaxf(m, h.log_prior[k]);
    float se = 0.f;
    for (int k = 0; k < h.K; ++k) se += __expf(h.log_prior[k] - m);
    if (si < h.K) lp_i = h.log_prior[si] - (m + __logf(se));
  }
  float s_rec = 0.f, s_ent = 0.f, s_tr = 0.f, s_init = 0.f, q0acc = 0.f, db2acc = 0.f;
  f32x4 gW2 = f32x4{0.f, 0.f, 0.f, 0.f}, gW1 = gW2;  // this wave's hidden block (hb = wave, HB <= 8)

  // this wave's block: window rows 16 w .. 16 w + 15 in every layer.  Stored rows (window rows ST_HALO ..
  // ST_HALO + ST_OWN - 1): l16 in [slo, shi)
  const int mlo = ST_HALO - 16 * wave, mhi = ST_HALO + ST_OWN - 16 * wave;  // in block-row units
  const int slo = max(0, mlo), shi = min(16, mhi);
  const bool nost = a.dbg & 1;
  int it = 0;
  for (; s < a.nstrip; s += gridDim.x) {
    const int64_t s0 = s * ST_OWN - ST_HALO;  // PCL row of window row 0
    const int64_t rb = s0 + 16 * wave;        // PCL row of this wave's block row 0
    {
      const int64_t nx = s + gridDim.x;
      px = load_x((nx < a.nstrip ? nx : s) * ST_OWN - ST_HALO);  // the next strip's x, in flight
    }
    // ---- enc_conv1 + ReLU for rows rb .. rb + 15 (h1e: owned rows) -> slot rows 1..16, row rb to the
    // previous wave's slot row 17, row rb + 15 to the next wave's slot row 0; the window's outer rows -1
    // and 128 (slot 0 row 0, slot 7 row 17) by waves 5 and 6 (SIMDs 1 and 2: no SIMD runs three blocks
    // twice as long as another)
    {
      f32x4 acc[4];
      pk_block(wE, sh.Xx + (16 * wave + 1) * ST_XLD, a.D, lg4, l16, acc);
      front_epi(acc, bE, rb, R, T, lg4, l16, slo, shi, a.h1e, slot + ST_LDW, nost, -1,
                wave > 0 ? sh.slot[wave - 1] + 17 * ST_LDW : nullptr, wave < 7 ? sh.slot[wave + 1] : nullptr);
      if (wave == 5 || wave == 6) {
        const bool lo = wave == 5;
        f32x4 acc2[4];
        pk_block(wE, sh.Xx + (lo ? 0 : 16 * 7 + 2) * ST_XLD, a.D, lg4, l16, acc2);
        front_epi(acc2, bE, lo ? s0 - 1 : s0 + 16 * 7 + 1, R, T, lg4, l16, 0, 0, a.h1e,
                  lo ? sh.slot[0] : sh.slot[7] + 2 * ST_LDW, true, lo ? 0 : 15);
      }
    }
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first strip: the image DMA
    lds_barrier();  // every slot's rows (and, first strip, every wave's share of the images)
    // ---- enc_conv2 + ReLU (h2e) + to_logits (logits) + softmax (q; all 16 rows -> Xq)
    {
      f32x4 acc[NB2][1];
#pragma unroll
      for (int nb = 0; nb < NB2; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<NB2, 1, 4, 3, ST_LDW, NW2>(sh.We2, slot, lg4, l16, acc, true);
      f32x4 y[NB2];
#pragma unroll
      for (int nb = 0; nb < NB2; ++nb) y[nb] = acc[nb][0];
      if constexpr (HTH > 0) kE.load(sh.Ee2, lg4, l16);
      tail_epi<NB2, true>(y, kE, rb, R, T, lg4, l16, slo, shi, a.H2, a.h2e, a.K, a.logits, a.q,
                          sh.Xq + (16 * wave + 2) * ST_XLD, nost);
    }
    lds_barrier();  // q of every block; everyone is done with Xx
    if (it == 0) stamp<PROF>(2);
    if constexpr (HTH > 0) {
      if (it == 0) {  // every wave read its constants into registers before this strip: the region is free
        float* hw = &sh.Wf[0][0];
#pragma unroll
        for (int j = 0; j < HNJ; ++j)
          if (tid + 512 * j < HNW) hw[tid + 512 * j] = hwv[j];
      }
    }
    // ---- composed dec_conv1 + ReLU for rows rb .. rb + 15 (g1: owned rows) -> slots, as enc_conv1
    {
      f32x4 acc[4];
      pk_block(wD, sh.Xq + (16 * wave + 1) * ST_XLD, a.K, lg4, l16, acc);
      if constexpr (PROF > 0) {
        if (it == 0) {
          asm volatile("s_nop 0" : : "v"(acc[3][3]));
          stamp<PROF>(10);
        }
      }
      front_epi(acc, bD, rb, R, T, lg4, l16, slo, shi, a.g1, slot + ST_LDW, nost, -1,
                wave > 0 ? sh.slot[wave - 1] + 17 * ST_LDW : nullptr, wave < 7 ? sh.slot[wave + 1] : nullptr);
      if (it == 0) stamp<PROF>(11);
      if (wave == 5 || wave == 6) {
        const bool lo = wave == 5;
        f32x4 acc2[4];
        pk_block(wD, sh.Xq + (lo ? 0 : 16 * 7 + 2) * ST_XLD, a.K, lg4, l16, acc2);
        front_epi(acc2, bD, lo ? s0 - 1 : s0 + 16 * 7 + 1, R, T, lg4, l16, 0, 0, a.g1,
                  lo ? sh.slot[0] : sh.slot[7] + 2 * ST_LDW, true, lo ? 0 : 15);
      }
    }
    lds_barrier();  // every slot's rows
    if (it == 0) stamp<PROF>(4);
    // ---- dec_conv2 + ReLU (g2) + to_params (par)
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<4, 1, 4, 3, ST_LDW, 64>(sh.Wd2, slot, lg4, l16, acc, true);
      f32x4 y[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) y[nb] = acc[nb][0];
      if constexpr (PROF > 0) {
        if (it == 0) {
          asm volatile("s_nop 0" : : "v"(y[3][3]));  // the loop's results are in
          stamp<PROF>(5);
        }
      }
      if constexpr (HTH > 0) kD.load(sh.Ed2, lg4, l16);
      tail_epi<4, false>(y, kD, rb, R, T, lg4, l16, slo, shi, 64, a.g2, a.P, a.par, nullptr, nullptr, nost);
    }
    if (it == 0) stamp<PROF>(6);
    // the next strip's x (Xx is free: every wave passed the barrier after its last read)
    {
      const int64_t nx = s + gridDim.x;
      store_x((nx < a.nstrip ? nx : s) * ST_OWN - ST_HALO, px);
    }
    if constexpr (HTH > 0) __syncthreads();  // + mu | logvar (HBM) of every block, for the head
    else lds_barrier();                      // Xx written; Xq and the slots free again
    if (it == 0) stamp<PROF>(3);
    if constexpr (HTH > 0) {
      // ================= fused ELBO head on window rows ST_HALO .. ST_HALO + ST_OWN (the last one = the
      // halo row whose log_A the last owned row's t -> t+1 term needs): head_coop.hip's phases, WR = 128
      StripHeadLds& hs = *reinterpret_cast<StripHeadLds*>(&sh.slot[0][0]);
      const StripHeadW<HTH>& hw = *reinterpret_cast<const StripHeadW<HTH>*>(&sh.Wf[0][0]);
      constexpr int LDL = StripHeadLds::LDL;
      const int K = h.K, U = h.U, D = h.D, KK = K * K;
      const int ldp = ld4(2 * D), ldxh = ld4(D), ldu = ld4(U);
      const int64_t r = s0 + ST_HALO + prow;
      const unsigned Tp = (unsigned)T + 2u;
      const unsigned rcl = (unsigned)(r < R ? r : R - 1);
      const int b = (int)(rcl / Tp);
      const int t = (int)(rcl - (unsigned)b * Tp) - 1;
      const bool valid = r < R && prow <= ST_OWN && t >= 0 && t < T;
      const bool own = prow < ST_OWN && r < R;
      const int64_t L = h.lengths[b];
      const bool m = valid && t < L;
      const float wgt = (valid && t >= 1 && t < L) ? 1.f : 0.f;  // pair (t-1, t) inside the length
      const float* qrow = sh.Xq + (ST_HALO + prow + 2) * ST_XLD;  // q | logits of the row
      float qv[HKP];
#pragma unroll
      for (int k = 0; k < HKP; ++k) qv[k] = (valid && k < K) ? qrow[k] : 0.f;
      const float qp = (valid && t >= 1 && si < K) ? qrow[si - ST_XLD] : 0.f;  // q[t-1][i]
      float qi = 0.f;
#pragma unroll
      for (int k = 0; k < HKP; ++k) qi = si == k ? qv[k] : qi;
      float mu[2], lv[2], xv[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = min(si + HKP * k, D - 1);
        mu[k] = h.par[(int64_t)rcl * ldp + c];
        lv[k] = h.par[(int64_t)rcl * ldp + D + c];
        xv[k] = h.x[(int64_t)rcl * ldxh + c];
      }
      const float uu = h.u[(int64_t)rcl * ldu + min(si, ldu - 1)];
      // ---- L: u' rows; dlgS's columns past K^2 zero
#pragma unroll
      for (int c = si; c < 8; c += HKP) hs.uS[prow * 8 + c] = c < U ? (valid ? uu : 0.f) : (c == U ? 1.f : 0.f);
      for (int i = tid; i < ST_WIN * LDL; i += 512)
        if (i % LDL >= KK) hs.dlgS[i] = 0.f;
      lds_barrier();
      // ---- A: transition logits lg^T = W2 relu(W1' u'^T) + b2, wave w = row block w (ij block 0: K^2 <= 16)
      {
        f32x4 lg;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int ij = 4 * lg4 + v;
          lg[v] = ij < KK ? h.b2[ij] : 0.f;
        }
        const float ub = hs.uS[(wave * 16 + l16) * 8 + lg4];
#pragma unroll 2
        for (int hb = 0; hb < HB; ++hb) {
          const float w1a = lg4 < U ? hw.W1S[(hb * 16 + l16) * 8 + lg4] : 0.f;
          f32x4 bb;
#pragma unroll
          for (int v = 0; v < 4; ++v) bb[v] = hw.W1S[(hb * 16 + 4 * lg4 + v) * 8 + U];
          const f32x4 w2v = *reinterpret_cast<const f32x4*>(&hw.W2S[l16 * HLDW2 + hb * 16 + 4 * lg4]);
          const f32x4 hc = mfma16x16x4(w1a, ub, bb);  // hid^T (h x rows), bias start
#pragma unroll
          for (int v = 0; v < 4; ++v) lg = mfma16x16x4(w2v[v], relu_f(hc[v]), lg);
        }
        *reinterpret_cast<f32x4*>(&hs.lgS[(wave * 16 + l16) * LDL + 4 * lg4]) = lg;
      }
      lds_barrier();
      // ---- B: log_softmax rows, transition term, d log_A -> d logits, recon NLL, entropy, init term
      float rsj = 0.f;
      {
        float la[HKP];
        float A_i = 0.f;
        const float* lr = &hs.lgS[prow * LDL + (si < K ? si : 0) * K];
        float mx = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < HKP; ++j) {
          la[j] = j < K ? lr[j] : 0.f;
          if (j < K) mx = fmaxf(mx, la[j]);
        }
        float se = 0.f;
#pragma unroll
        for (int j = 0; j < HKP; ++j)
          if (j < K) se += __expf(la[j] - mx);
        const float ls = mx + __logf(se);
#pragma unroll
        for (int j = 0; j < HKP; ++j)
          if (j < K) la[j] -= ls;
#pragma unroll
        for (int j = 0; j < HKP; ++j)
          if (j < K) A_i = fmaf(qv[j], la[j], A_i);
        if (si >= K) A_i = 0.f;
        float c[HKP];
#pragma unroll
        for (int j = 0; j < HKP; ++j) c[j] = (j < K && si < K) ? qp * la[j] : 0.f;
        rsj = row4_reduce_scatter(c, si);
        if (own && si < K) s_tr = fmaf(wgt * qp, A_i, s_tr);
        hs.aS[prow * HKP + si] = A_i;
        if (si == 0) hs.wS[prow] = wgt;
        if (hgrad && si < K) {
          float qs = 0.f;
#pragma unroll
          for (int j = 0; j < HKP; ++j)
            if (j < K) qs += qv[j];
          const float g = own ? cpri * wgt * qp : 0.f;
          const float rs = g * qs;
          float* dl = &hs.dlgS[prow * LDL + si * K];
#pragma unroll
          for (int j = 0; j < HKP; ++j)
            if (j < K) dl[j] = g * qv[j] - __expf(la[j]) * rs;
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int ch = si + HKP * k;
        float dmu = 0.f, dlv = 0.f;
        if (own && m && ch < D) {
          const float ev = __expf(lv[k]);
          const float var = ev < 1e-8f ? 1e-8f : ev;  // clamp(min=1e-8), NaN stays NaN
          const float df = mu[k] - xv[k];
          const float r2 = df * df / var;
          s_rec += 0.5f * (__logf(6.2831855f * var) + r2);
          dmu = df / var * inv_n;
          dlv = (ev >= 1e-8f) ? 0.5f * (1.f - r2) * inv_n : 0.f;
        }
        if (hgrad && own && ch < D) {
          h.dpar[r * ldp + ch] = dmu;
          h.dpar[r * ldp + D + ch] = dlv;
        }
      }
      if (hgrad && own && 2 * D + si < ldp) h.dpar[r * ldp + 2 * D + si] = 0.f;
      {
        const float lgv = (valid && si < K) ? qrow[4 + si] : 0.f;
        const float mx = row4_max(si < K ? lgv : -__builtin_inff());
        const float lse = mx + __logf(row4_sum(si < K ? __expf(lgv - mx) : 0.f));
        const float f = row4_sum(si < K ? qi * (lgv - lse) : 0.f);
        if (own && m && si == 0) s_ent -= f;
        if (hgrad && own) h.dlx[r * HKP + si] = (m && si < K) ? cent * qi * ((lgv - lse) - f) : 0.f;
      }
      if (own && valid && t == 0 && si < K) {
        s_init = fmaf(qi, lp_i, s_init);
        q0acc += qi;
      }
      lds_barrier();  // dlgS, aS, wS of every row
      // ---- B2: dq
      if (hgrad && own) {
        float v = cpri * (wgt * rsj + hs.wS[prow + 1] * hs.aS[(prow + 1) * HKP + si]);
        if (valid && t == 0) v = fmaf(cpri, lp_i, v);
        h.dqx[r * HKP + si] = (valid && si < K) ? v : 0.f;
      }
      // ---- C: MLP backward, wave w = hidden block w
      if (hgrad) {
        if (wave == 0) {  // db2: column sums of dlg, ij = l16
#pragma unroll 8
          for (int k = 0; k < ST_WIN / 4; ++k) db2acc += hs.dlgS[(lg4 * (ST_WIN / 4) + k) * LDL + l16];
        }
        if (wave < HB) {
          const int hb = wave;
          const float w1 = hw.W1S[(hb * 16 + l16) * 8 + lg4];
          const float bb1 = hw.W1S[(hb * 16 + l16) * 8 + U];
          float w2c[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) w2c[s4] = hw.W2S[(4 * s4 + lg4) * HLDW2 + hb * 16 + l16];
          const int SD = (KK + 3) / 4;
#pragma unroll 2
          for (int rb = 0; rb < ST_WIN / 16; ++rb) {
            const float ua = lg4 < U ? hs.uS[(rb * 16 + l16) * 8 + lg4] : 0.f;
            float dla[4], dlt[4], ubv[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
              dla[s4] = s4 < SD ? hs.dlgS[(rb * 16 + l16) * LDL + 4 * s4 + lg4] : 0.f;
              const int row = rb * 16 + 4 * lg4 + s4;
              dlt[s4] = hs.dlgS[row * LDL + l16];
              const float uv = hs.uS[row * 8 + (l16 & 7)];
              ubv[s4] = l16 < 8 ? uv : 0.f;
            }
            const f32x4 hh = mfma16x16x4(ua, w1, f32x4{bb1, bb1, bb1, bb1});  // (rows x h), bias start
            f32x4 dh = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
              if (s4 < SD) dh = mfma16x16x4(dla[s4], w2c[s4], dh);  // dlg @ W2
            f32x4 hr, dm;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              hr[v] = relu_f(hh[v]);
              dm[v] = hh[v] > 0.f ? dh[v] : 0.f;
            }
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
              gW2 = mfma16x16x4(dlt[s4], hr[s4], gW2);  // dlg^T hid
              gW1 = mfma16x16x4(dm[s4], ubv[s4], gW1);  // dhid^T u'
            }
          }
        }
      }
      lds_barrier();  // the head's LDS reads are done before the next strip writes the slots and Xq
    }
    ++it;
  }
  if constexpr (HTH > 0) {
    // ---- head epilogue: loss partials, q0 / db2 sums, weight-gradient partials (fixed order), as head_coop
    StripHeadLds& hs = *reinterpret_cast<StripHeadLds*>(&sh.slot[0][0]);
    double ds[4] = {(double)s_rec, (double)s_init, (double)s_tr, (double)s_ent};
#pragma unroll
    for (int k = 0; k < 4; ++k) ds[k] = wave_sum_dpp(ds[k]);
    q0acc += __shfl_xor(q0acc, 4);
    q0acc += __shfl_xor(q0acc, 8);
    q0acc += xor16(q0acc);
    q0acc += xor32(q0acc);
    db2acc += xor16(db2acc);
    db2acc += xor32(db2acc);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) hs.red[wave][k] = ds[k];
    if (lane < HKP) hs.q0w[wave][lane] = q0acc;
    __syncthreads();
    const int K = h.K, KK = K * K;
    if (tid < 4) {
      double v = 0.0;
      for (int w = 0; w < 8; ++w) v += hs.red[w][tid];
      h.part[blockIdx.x * 4 + tid] = v;
    }
    if (hgrad) {
      if (tid < K) {
        float v = 0.f;
        for (int w = 0; w < 8; ++w) v += hs.q0w[w][tid];
        h.slab_q0[(int64_t)blockIdx.x * K + tid] = v;
      }
      if (wave == 0 && lane < 16 && lane < KK) h.slab_b2[(int64_t)blockIdx.x * KK + lane] = db2acc;
      if (wave < HB) {
        float* sW2 = h.slab_W2 + (int64_t)blockIdx.x * KK * HTH;
        float* sW1 = h.slab_W1 + (int64_t)blockIdx.x * HTH * h.U;
        float* sb1 = h.slab_b1 + (int64_t)blockIdx.x * HTH;
        const int hb = wave;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int ij = 4 * lg4 + v;
          if (ij < KK) sW2[ij * HTH + hb * 16 + l16] = gW2[v];
          const int hh = hb * 16 + 4 * lg4 + v;  // gW1' lane -> (h, c' = l16); c' == U is db1
          if (l16 < h.U) sW1[hh * h.U + l16] = gW1[v];
          else if (l16 == h.U) sb1[hh] = gW1[v];
        }
      }
    }
  }
  if constexpr (PROF > 0) {
    __syncthreads();
    stamp<PROF>(7);
    if constexpr (PROF > 0) { if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 14] = __builtin_amdgcn_s_memtime(); }
    if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 8] = (unsigned long long)it;
  }
}

static int prof_on() {
  static const int v = prof_env("VQHMM_STRIP_PROF");
  return v;
}

// ---------------------------------------------------------------------------------------------
// Backward strip: to_params dgrad (1x1, mask g2) -> dec_conv2 dgrad (mask g1) -> composed dec_conv1
// dgrad + softmax backward + to_logits dgrad (mask h2) -> enc_conv2 dgrad (mask h1) in ONE launch
// (VQ_VAE_HMM_fixed.py:80-90 / :38-41 backward).  Wave w owns the window's block w: it computes the
// 1x1 front for the 18 rows its dec_conv2 dgrad reads (dpar and the g2 mask come from HBM, so they are
// exact at the window edges too), then dg1 goes through LDS (aliasing the per-wave slots) to the
// dec_conv1 dgrad, and dh2 through LDS to the enc_conv2 dgrad: three workgroup barriers per strip;
// rows >= 2 from the window edges are exact and stored.  Same MFMA sequences and epilogue
// arithmetic as the pair launches (conv2f_kernel's front / main conv, conv2g_kernel's pair).
struct StripBwdArgs {
  int64_t R;
  int T, ldp;                      // ldp = ld4(2D): dpar row stride (<= 16)
  const float* dpar;               // PCL (R, ldp): the head's gradient of mu | logvar
  const float *g2, *g1, *h1e;      // the ReLU masks (PCL, 64 channels)
  const float *img_pd, *img_d2, *img_c1, *img_e2;  // dgrad images: [1][64][24], [3][64][72], [3][16][72], [3][64][40]
  const float* gscale;             // device scale of dpar (null: 1)
  float *dg2, *dg1, *dh1;
  int64_t nstrip;
};

namespace {
struct StripBwdLds {
  float Wd2[3 * 64 * ST_LDW];    // dec_conv2 dgrad image
  float We2[3 * 64 * SB_LDE];    // enc_conv2 dgrad image (32 input channels)
  float Wc1[3 * 16 * ST_LDW];    // composed dec_conv1 dgrad image (K <= 4 outputs of 16)
  float slot[8][18 * ST_LDW];    // per wave: dg2 rows rb - 1 .. rb + 16; then, all waves: dg1 rows s0 - 1 ..
  float Dh2[(ST_WIN + 2) * SB_LDE];  // dh2 rows s0 - 1 .. s0 + 128
};
static_assert(8 * 18 * ST_LDW >= (ST_WIN + 2) * ST_LDW, "dg1 rows alias the slots");

}  // namespace

template <int PROF>
__global__ __launch_bounds__(512) void strip_bwd_kernel(StripBwdArgs a, ConvArgs f) {
  extern __shared__ float4 smem4[];
  StripBwdLds& sh = *reinterpret_cast<StripBwdLds*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int64_t R = a.R;
  const int T = a.T;
  float* slot = sh.slot[wave];
  float* D1 = &sh.slot[0][0];  // dg1 rows s0 - 1 .. s0 + 128 (after the slots' last read)

  stamp<PROF>(0);
  // ---- once: the 1x1 front's weights (registers), then the images by LDS DMA (waited for before the
  // first dec_conv2 dgrad)
  float wP[4][4];  // A operand of the 1x1 front: image[n = nb*16 + l16][k = 4 lg4 + e]
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const float4 w4 = *reinterpret_cast<const float4*>(a.img_pd + (nb * 16 + l16) * ST_LDF + 4 * lg4);
    wP[nb][0] = w4.x; wP[nb][1] = w4.y; wP[nb][2] = w4.z; wP[nb][3] = w4.w;
  }
  const float psc = a.gscale ? *a.gscale : 1.0f;
  {
    constexpr int N1 = 3 * 64 * ST_LDW / 4, N2 = 3 * 64 * SB_LDE / 4, N3 = 3 * 16 * ST_LDW / 4;
    constexpr int C1 = (N1 + 63) / 64, C2 = (N2 + 63) / 64, C3 = (N3 + 63) / 64;
    for (int c = wave; c < C1 + C2 + C3; c += 8) {
      const int k = c < C1 ? 0 : c < C1 + C2 ? 1 : 2;
      const int cc = k == 0 ? c : k == 1 ? c - C1 : c - C1 - C2;
      const int i = cc * 64 + lane, n = k == 0 ? N1 : k == 1 ? N2 : N3;
      const float* src = k == 0 ? a.img_d2 : k == 1 ? a.img_e2 : a.img_c1;
      float* dst = k == 0 ? sh.Wd2 : k == 1 ? sh.We2 : sh.Wc1;
      if (i < n) dma16(src + 4 * i, dst + cc * 256);
    }
  }
  stamp<PROF>(1);

  const int mlo = ST_HALO - 16 * wave, mhi = ST_HALO + ST_OWN - 16 * wave;
  const int slo = max(0, mlo), shi = min(16, mhi);
  int it = 0;
  for (int64_t s = blockIdx.x; s < a.nstrip; s += gridDim.x) {
    const int64_t s0 = s * ST_OWN - ST_HALO;
    const int64_t rb = s0 + 16 * wave;
    // ---- to_params dgrad (1x1, x scale, mask g2) for rows rb .. rb + 15 -> dg2, slot rows 1..16, the
    // neighbours' halo rows (17 / 0); the window's outer rows -1 / 128 by waves 5 / 6 (as the forward strip)
    {
      auto ld_dpar = [&](int64_t r) {  // row r, channels 4 lg4 .. (x_mask: rows outside / pad channels 0)
        const int64_t rc = r < 0 ? 0 : (r >= R ? R - 1 : r);
        const float4 v = *reinterpret_cast<const float4*>(a.dpar + rc * a.ldp + min(4 * lg4, a.ldp - 4));
        return (r >= 0 && r < R && 4 * lg4 < a.ldp) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      };
      auto front = [&](int64_t r0, float4 (&m)[4], const float4 x, f32x4 (&acc)[4]) {
        const float b[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma16x16x4(wP[nb][e], b[e], acc[nb]);
      };
      const bool extra = wave == 5 || wave == 6;
      const int64_t re = wave == 5 ? s0 - 1 : s0 + 16 * 7 + 1;  // the extra block's row 0
      float4 mA[4], mB[4], xA, xB = make_float4(0.f, 0.f, 0.f, 0.f);
      load_mask(a.g2, rb, R, lg4, l16, mA);
      xA = ld_dpar(rb + l16);
      if (extra) {
        load_mask(a.g2, re, R, lg4, l16, mB);
        xB = ld_dpar(re + l16);
      }
      f32x4 acc[4];
      front(rb, mA, xA, acc);
      mask_epi(acc, mA, psc, rb, R, T, lg4, l16, slo, shi, a.dg2, slot + ST_LDW, ST_LDW, -1,
               wave > 0 ? sh.slot[wave - 1] + 17 * ST_LDW : nullptr, wave < 7 ? sh.slot[wave + 1] : nullptr);
      if (extra) {
        f32x4 acc2[4];
        front(re, mB, xB, acc2);
        mask_epi(acc2, mB, psc, re, R, T, lg4, l16, 0, 0, a.dg2, wave == 5 ? sh.slot[0] : sh.slot[7] + 2 * ST_LDW,
                 ST_LDW, wave == 5 ? 0 : 15);
      }
    }
    float4 m1[4];
    load_mask(a.g1, rb, R, lg4, l16, m1);
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first strip: the image DMA
    lds_barrier();  // every slot's rows (and, first strip, every wave's share of the images)
    // ---- dec_conv2 dgrad (mask g1) -> dg1 (registers, HBM)
    f32x4 d1[4];
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<4, 1, 4, 3, ST_LDW, 64>(sh.Wd2, slot, lg4, l16, acc, true);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) d1[nb] = acc[nb][0];
      mask_epi(d1, m1, 1.0f, rb, R, T, lg4, l16, slo, shi, a.dg1, nullptr, 0);
    }
    lds_barrier();  // every slot read
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) *reinterpret_cast<f32x4*>(D1 + (16 * wave + 1 + l16) * ST_LDW + nb * 16 + 4 * lg4) = d1[nb];
    float4 m2[4];
    load_mask(a.h1e, rb, R, lg4, l16, m2);
    lds_barrier();  // dg1 of every block
    if (it == 0) stamp<PROF>(2);
    // ---- composed dec_conv1 dgrad + softmax backward + to_logits dgrad (mask h2): dqd, dlog, dh2 (HBM),
    // dh2 of all 16 rows -> Dh2 (conv2g_kernel's front, conv2_epilogue ACT 3)
    {
      f32x4 acc1[1][1] = {{f32x4{0.f, 0.f, 0.f, 0.f}}};
      c2_mfma_tile<1, 1, 4, 3, ST_LDW, 16>(sh.Wc1, D1 + 16 * wave * ST_LDW, lg4, l16, acc1, true);
      const float zb1[1][4] = {}, tw1[1][4] = {};
      const float4 aux1[1][1] = {};
      const float fsc = f.scale ? *f.scale : 1.0f;
      conv2_epilogue<1, 1, 3>(f, rb, 0, lg4, l16, acc1, aux1, zb1, tw1, f32x4{0.f, 0.f, 0.f, 0.f}, fsc, false, slo,
                              shi, sh.Dh2 + (16 * wave + 1) * SB_LDE, SB_LDE);
    }
    lds_barrier();  // dh2 of every block
    if (it == 0) stamp<PROF>(3);
    // ---- enc_conv2 dgrad (mask h1) -> dh1
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<4, 1, 2, 3, SB_LDE, 64>(sh.We2, sh.Dh2 + 16 * wave * SB_LDE, lg4, l16, acc, true);
      f32x4 y[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) y[nb] = acc[nb][0];
      mask_epi(y, m2, 1.0f, rb, R, T, lg4, l16, slo, shi, a.dh1, nullptr, 0);
    }
    // no barrier: the next strip writes the slots (dg1, last read before the barrier above) and Dh2
    // only after its own first two barriers
    ++it;
  }
  if constexpr (PROF > 0) {
    __syncthreads();
    stamp<PROF>(7);
    if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 8] = (unsigned long long)it;
  }
}

bool strip_bwd_supported(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2) {
  return pd.R > 0 && pd.R < (1ll << 31) && pd.ks == 1 && pd.act == 2 && pd.Wimg && pd.aux && pd.out && pd.N == 64 &&
         pd.Kc >= 1 && pd.Kc <= 16 && !pd.src_cf && !pd.bias &&
         d2.src == pd.out && d2.ks == 3 && d2.act == 2 && d2.Wimg && d2.aux && d2.out && d2.Kc == 64 && d2.N == 64 &&
         !d2.bias && !d2.scale &&
         f.src == d2.out && f.act == 3 && f.ks == 3 && f.Wimg && f.Kc == 64 && f.N >= 1 && f.N <= 4 && f.lb_dh &&
         f.lb_C > 16 && f.lb_C <= 32 && ld4(f.lb_C) == 32 && !f.bias && !f.out_cf &&
         e2.src == f.lb_dh && e2.ks == 3 && e2.act == 2 && e2.Wimg && e2.aux && e2.out && e2.Kc == f.lb_C &&
         e2.N == 64 && !e2.bias && !e2.scale && !e2.tW && !e2.out_cf;
}

int launch_strip_bwd(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2, hipStream_t s) {
  if (!strip_bwd_supported(pd, d2, f, e2)) return VQHMM_EUNSUPPORTED;
  StripBwdArgs a{};
  a.R = pd.R; a.T = pd.T; a.ldp = ld4(pd.Kc);
  a.dpar = pd.src; a.g2 = pd.aux; a.g1 = d2.aux; a.h1e = e2.aux;
  a.img_pd = pd.Wimg; a.img_d2 = d2.Wimg; a.img_c1 = f.Wimg; a.img_e2 = e2.Wimg;
  a.gscale = pd.scale;
  a.dg2 = pd.out; a.dg1 = d2.out; a.dh1 = e2.out;
  a.nstrip = cdiv(pd.R, ST_OWN);
  const unsigned grid = (unsigned)(a.nstrip < 256 ? a.nstrip : 256);
  if (prof_on()) strip_bwd_kernel<1><<<grid, 512, sizeof(StripBwdLds), s>>>(a, f);
  else strip_bwd_kernel<0><<<grid, 512, sizeof(StripBwdLds), s>>>(a, f);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

static StripFwdArgs strip_fwd_args(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2) {
  StripFwdArgs a{};
  a.R = e1.R; a.T = e1.T; a.D = e1.Kc; a.H2 = e2.N; a.K = e2.C2; a.P = d2.C2;
  a.xp = e1.src;
  a.img_e1 = e1.Wimg; a.img_d1 = d1.Wimg; a.img_e2 = e2.Wimg; a.img_d2 = d2.Wimg;
  a.b_e1 = e1.bias; a.b_e2 = e2.bias; a.b_d1 = d1.bias; a.b_d2 = d2.bias;
  a.tWl = e2.tW; a.tbl = e2.tb; a.tWp = d2.tW; a.tbp = d2.tb;
  a.h1e = e1.out; a.h2e = e2.out; a.logits = e2.t_out; a.q = e2.q_out; a.g1 = d1.out; a.g2 = d2.out; a.par = d2.t_out;
  a.nstrip = cdiv(e1.R, ST_OWN);
  static const int dbg = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_STRIP_DBG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
  return a;
}

bool strip_fwd_supported(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2) {
  auto relu3 = [](const ConvArgs& a) { return a.ks == 3 && a.act == 1 && !a.src_cf && a.Wimg && a.out && !a.out_cf; };
  return relu3(e1) && relu3(e2) && relu3(d1) && relu3(d2) && e1.R > 0 && e1.R < (1ll << 31) &&
         e1.Kc >= 1 && 3 * e1.Kc <= 16 && e1.N == 64 &&                                   // packed front
         e2.src == e1.out && e2.Kc == 64 && e2.N >= 1 && e2.N <= 32 &&                    // 64 -> H2 (LDS)
         e2.C2 >= 1 && e2.C2 <= 4 && e2.t_out && e2.q_out && !e2.q_cf && !e2.reg_out && !e2.t_cf0 &&
         d1.src == e2.q_out && d1.Kc == e2.C2 && 3 * d1.Kc <= 16 && d1.N == 64 &&         // packed front
         d2.src == d1.out && d2.Kc == 64 && d2.N == 64 && d2.C2 >= 1 && d2.C2 <= 16 && d2.t_out && !d2.t_cf0 &&
         !d2.q_out && !d2.q_cf && !d2.reg_out;
}

int strip_prof_copy(uint64_t* out, int64_t n) { return prof_copy(out, n); }

bool strip_head_supported(const HeadArgs& h) {
  return h.K >= 1 && h.K <= 4 && h.U >= 1 && h.U <= 4 && (h.TH == 64 || h.TH == 128) && h.D >= 1 && h.D <= 8 &&
         h.R < (1ll << 31);
}

int strip_fwd_grid(int64_t R) {
  const int64_t n = cdiv(R, ST_OWN);
  return (int)(n < 256 ? (n > 0 ? n : 1) : 256);
}

int launch_strip_fwd(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2, const HeadArgs* h,
                     hipStream_t s) {
  if (!strip_fwd_supported(e1, e2, d1, d2)) return VQHMM_EUNSUPPORTED;
  if (h && (!strip_head_supported(*h) || h->K != e2.C2 || h->R != e1.R || h->D != e1.Kc)) return VQHMM_EUNSUPPORTED;
  const StripFwdArgs a = strip_fwd_args(e1, e2, d1, d2);
  const unsigned grid = (unsigned)strip_fwd_grid(e1.R);
  const HeadArgs hv = h ? *h : HeadArgs{};
  const int hth = h ? h->TH : 0;
#define VQHMM_SF(NB2, P, HT) strip_fwd_kernel<NB2, P, HT><<<grid, 512, sizeof(StripFwdLds<NB2>), s>>>(a, hv)
#define VQHMM_SF_H(NB2, P) \
  if (hth == 128) VQHMM_SF(NB2, P, 128); else if (hth == 64) VQHMM_SF(NB2, P, 64); else VQHMM_SF(NB2, P, 0);
  const bool prof = prof_on() != 0;
  if (c2_nb(e2.N) == 1) {
    if (prof) { VQHMM_SF_H(1, 1) } else { VQHMM_SF_H(1, 0) }
  } else {
    if (prof) { VQHMM_SF_H(2, 1) } else { VQHMM_SF_H(2, 0) }
  }
#undef VQHMM_SF_H
#undef VQHMM_SF
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm

