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

#include "conv2_dev.h"
#include "prof.h"

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
constexpr int ST_WIN = 128;                    // window rows: 8 MFMA row blocks, one per wave
constexpr int ST_HALO = 2;                     // inexact rows on each side
constexpr int ST_OWN = ST_WIN - 2 * ST_HALO;   // rows a strip stores
constexpr int ST_XR = ST_WIN + 4;              // rows of the shared x / q buffers (s0 - 2 .. s0 + 129)
constexpr int ST_XLD = 8;                      // their row stride
constexpr int ST_LDW = 72;                     // c2_ldx(64): 64-channel slots and weight images
constexpr int ST_LDF = 24;                     // the prologue's packed-front image row stride


template <int NB2>
struct StripFwdLds {
  static constexpr int NW2 = 16 * NB2;
  float We2[3 * NW2 * ST_LDW];  // enc_conv2 image
  float Wd2[3 * 64 * ST_LDW];   // dec_conv2 image
  float Wf[2][3 * 64 * 8];      // enc_conv1 / dec_conv1 images, channels 0..7 ([tap][n][8])
  float Ee2[NW2 * 17 + 16];     // enc_conv2 bias | to_logits weight (16 x NW2) | bias
  float Ed2[64 * 17 + 16];      // dec_conv2 bias | to_params weight (16 x 64) | bias
  float bf[2][64];              // enc_conv1 / dec_conv1 bias
  float Xx[ST_XR * ST_XLD];     // x rows s0 - 2 .. s0 + 129
  float Xq[ST_XR * ST_XLD];     // q rows s0 - 2 .. s0 + 129 (the 2 + 2 outer rows stay zero)
  float slot[8][18 * ST_LDW];   // per wave: the 64-wide conv's 18 input rows rb - 1 .. rb + 16
};

// row_bt's validity test with 32-bit arithmetic (R < 2^31): PCL row r is a sequence position
__device__ __forceinline__ bool row_valid(int64_t r, int64_t R, int T) {
  if (r < 0 || r >= R) return false;
  const unsigned Tp = (unsigned)T + 2u, m = (unsigned)r % Tp;
  return m >= 1u && m <= (unsigned)T;
}

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
// rows l16 in [slo, shi) are stored to out (PCL, 64 channels); every row goes to the LDS slot rows xs.
__device__ __forceinline__ void front_epi(f32x4 (&acc)[4], const f32x4 (&bias)[4], int64_t r0, int64_t R, int T,
                                          int lg4, int l16, int slo, int shi, float* out, float* xs,
                                          bool nostore) {
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
    *reinterpret_cast<f32x4*>(xs + l16 * ST_LDW + nb * 16 + 4 * lg4) = y;
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
    if (c0 < ST_XLD) *reinterpret_cast<f32x4*>(xq + l16 * ST_XLD + c0) = qv;
  }
}

// element i of a [bias (NW) | tail weight (16 x NW) | tail bias (16)] block
template <int NW>
__device__ __forceinline__ float es_val(const float* bias, int N, const float* tW, const float* tb, int C2, int i) {
  if (i < NW) return i < N ? bias[i] : 0.f;
  if (i < 17 * NW) {
    const int j = i - NW, c2 = j / NW, n = j - c2 * NW;
    return (c2 < C2 && n < N) ? tW[(int64_t)c2 * N + n] : 0.f;
  }
  const int c2 = i - 17 * NW;
  return c2 < C2 ? tb[c2] : 0.f;
}

__device__ __forceinline__ void dma16(const float* src, float* dst) {
  __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(src), (__attribute__((address_space(3))) void*)dst,
                                   16, 0, 0);
}
}  // namespace

template <int NB2, int PROF>
__global__ __launch_bounds__(512) void strip_fwd_kernel(StripFwdArgs a) {
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

  stamp<PROF>(0);
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
#pragma unroll
  for (int j = 0; j < NCJ; ++j) {
    const int i = tid + 512 * j;
    float v = 0.f;
    if (i < NE) v = es_val<NW2>(a.b_e2, a.H2, a.tWl, a.tbl, a.K, i);
    else if (i < NE + ND) v = es_val<64>(a.b_d2, 64, a.tWp, a.tbp, a.P, i - NE);
    else if (i < NC) v = (i - NE - ND < 64 ? a.b_e1 : a.b_d1)[(i - NE - ND) & 63];
    cv[j] = v;
  }
  {
    constexpr int N1 = 3 * NW2 * ST_LDW / 4, N2 = 3 * 64 * ST_LDW / 4;  // float4s of each image
    constexpr int C1 = (N1 + 63) / 64, C2 = (N2 + 63) / 64;              // one wave instruction = 1 KB
    for (int c = wave; c < C1 + C2; c += 8) {
      const bool first = c < C1;
      const int cc = first ? c : c - C1;
      const int i = cc * 64 + lane;
      if (i < (first ? N1 : N2)) dma16((first ? a.img_e2 : a.img_d2) + 4 * i, (first ? sh.We2 : sh.Wd2) + cc * 256);
    }
  }
  static_assert(offsetof(S, Ed2) == offsetof(S, Ee2) + NE * 4 && offsetof(S, bf) == offsetof(S, Ed2) + ND * 4,
                "constant blocks must be contiguous");
#pragma unroll
  for (int j = 0; j < NCJ; ++j)
    if (tid + 512 * j < NC) sh.Ee2[tid + 512 * j] = cv[j];
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
  TailConsts<NB2> kE;
  TailConsts<4> kD;
  kE.load(sh.Ee2, lg4, l16);
  kD.load(sh.Ed2, lg4, l16);

  // this wave's block: window rows 16 w .. 16 w + 15.  Stored rows (window rows ST_HALO .. ST_HALO +
  // ST_OWN - 1): the 64-wide convs' l16 range; the fronts' block A (rows 16w - 1 + l16) stores rows
  // 16w .. 16w + 14, block B (rows 16w + 1 + l16) row 16w + 15
  const int mlo = ST_HALO - 16 * wave, mhi = ST_HALO + ST_OWN - 16 * wave;  // in block-row units
  const int slo = max(0, mlo), shi = min(16, mhi);
  const int alo = max(1, mlo + 1), ahi = min(16, mhi + 1);
  const bool bown = 15 >= mlo && 15 < mhi;
  const bool nost = a.dbg & 1;
  int it = 0;
  for (; s < a.nstrip; s += gridDim.x) {
    const int64_t s0 = s * ST_OWN - ST_HALO;  // PCL row of window row 0
    const int64_t rb = s0 + 16 * wave;        // PCL row of this wave's block row 0
    {
      const int64_t nx = s + gridDim.x;
      px = load_x((nx < a.nstrip ? nx : s) * ST_OWN - ST_HALO);  // the next strip's x, in flight
    }
    // ---- enc_conv1 + ReLU for rows rb - 1 .. rb + 16 (h1e: owned rows) -> slot
    {
      f32x4 acc[4], acc2[4];
      pk_block(wE, sh.Xx + (16 * wave) * ST_XLD, a.D, lg4, l16, acc);
      pk_block(wE, sh.Xx + (16 * wave + 2) * ST_XLD, a.D, lg4, l16, acc2);
      front_epi(acc, bE, rb - 1, R, T, lg4, l16, alo, ahi, a.h1e, slot, nost);
      front_epi(acc2, bE, rb + 1, R, T, lg4, l16, bown ? 14 : 16, bown ? 15 : 16, a.h1e, slot + 2 * ST_LDW, nost);
    }
    if (it == 0) {  // the first strip: every wave's share of the image DMA has landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    } else {
      __builtin_amdgcn_wave_barrier();
    }
    // ---- enc_conv2 + ReLU (h2e) + to_logits (logits) + softmax (q; all 16 rows -> Xq)
    {
      f32x4 acc[NB2][1];
#pragma unroll
      for (int nb = 0; nb < NB2; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<NB2, 1, 4, 3, ST_LDW, NW2>(sh.We2, slot, lg4, l16, acc, true);
      f32x4 y[NB2];
#pragma unroll
      for (int nb = 0; nb < NB2; ++nb) y[nb] = acc[nb][0];
      tail_epi<NB2, true>(y, kE, rb, R, T, lg4, l16, slo, shi, a.H2, a.h2e, a.K, a.logits, a.q,
                          sh.Xq + (16 * wave + 2) * ST_XLD, nost);
    }
    lds_barrier();  // q of every block; everyone is done with Xx
    if (it == 0) stamp<PROF>(2);
    // ---- composed dec_conv1 + ReLU for rows rb - 1 .. rb + 16 (g1: owned rows) -> slot
    {
      f32x4 acc[4], acc2[4];
      pk_block(wD, sh.Xq + (16 * wave) * ST_XLD, a.K, lg4, l16, acc);
      pk_block(wD, sh.Xq + (16 * wave + 2) * ST_XLD, a.K, lg4, l16, acc2);
      if constexpr (PROF > 0) {
        if (it == 0) {
          asm volatile("s_nop 0" : : "v"(acc[3][3]), "v"(acc2[3][3]));
          stamp<PROF>(10);
        }
      }
      front_epi(acc, bD, rb - 1, R, T, lg4, l16, alo, ahi, a.g1, slot, nost);
      if (it == 0) stamp<PROF>(11);
      front_epi(acc2, bD, rb + 1, R, T, lg4, l16, bown ? 14 : 16, bown ? 15 : 16, a.g1, slot + 2 * ST_LDW, nost);
    }
    __builtin_amdgcn_wave_barrier();
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
      tail_epi<4, false>(y, kD, rb, R, T, lg4, l16, slo, shi, 64, a.g2, a.P, a.par, nullptr, nullptr, nost);
    }
    if (it == 0) stamp<PROF>(6);
    // the next strip's x (Xx is free: every wave passed the barrier after its last read)
    {
      const int64_t nx = s + gridDim.x;
      store_x((nx < a.nstrip ? nx : s) * ST_OWN - ST_HALO, px);
    }
    lds_barrier();  // Xx written; Xq and the slots free again
    if (it == 0) stamp<PROF>(3);
    ++it;
  }
  if constexpr (PROF > 0) {
    __syncthreads();
    stamp<PROF>(7);
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
constexpr int SB_LDE = 40;  // c2_ldx(32): enc_conv2's dgrad input rows (dh2) and its image

struct StripBwdLds {
  float Wd2[3 * 64 * ST_LDW];    // dec_conv2 dgrad image
  float We2[3 * 64 * SB_LDE];    // enc_conv2 dgrad image (32 input channels)
  float Wc1[3 * 16 * ST_LDW];    // composed dec_conv1 dgrad image (K <= 4 outputs of 16)
  float slot[8][18 * ST_LDW];    // per wave: dg2 rows rb - 1 .. rb + 16; then, all waves: dg1 rows s0 - 1 ..
  float Dh2[(ST_WIN + 2) * SB_LDE];  // dh2 rows s0 - 1 .. s0 + 128
};
static_assert(8 * 18 * ST_LDW >= (ST_WIN + 2) * ST_LDW, "dg1 rows alias the slots");

// conv2_epilogue's ACT = 2 arithmetic (scale, no bias, ReLU-backward mask, pad rows 0) on a 64-wide
// block: rows r0 + l16, stored (PCL, 64 channels) for l16 in [slo, shi), optionally to LDS rows xs
__device__ __forceinline__ void mask_epi(f32x4 (&acc)[4], const float4 (&aux)[4], float sc, int64_t r0, int64_t R,
                                         int T, int lg4, int l16, int slo, int shi, float* out, float* xs, int xld) {
  const int64_t r = r0 + l16;
  const bool valid = row_valid(r, R, T);
  const bool st = l16 >= slo && l16 < shi && r < R;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const float av[4] = {aux[nb].x, aux[nb].y, aux[nb].z, aux[nb].w};
    f32x4 y;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float yy = acc[nb][v] * sc + 0.f;
      yy = av[v] > 0.f ? yy : 0.f;
      y[v] = valid ? yy : 0.f;
    }
    acc[nb] = y;
    if (st) *reinterpret_cast<f32x4*>(out + r * 64 + nb * 16 + 4 * lg4) = y;
    if (xs) *reinterpret_cast<f32x4*>(xs + l16 * xld + nb * 16 + 4 * lg4) = y;
  }
}

// the 64-channel mask rows r0 + l16 of a block (clamped into [0, R): rows outside are not stored)
__device__ __forceinline__ void load_mask(const float* m, int64_t r0, int64_t R, int lg4, int l16, float4 (&aux)[4]) {
  int64_t r = r0 + l16;
  r = r < 0 ? 0 : (r >= R ? R - 1 : r);
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) aux[nb] = *reinterpret_cast<const float4*>(m + r * 64 + nb * 16 + 4 * lg4);
}
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
  const int alo = max(1, mlo + 1), ahi = min(16, mhi + 1);
  const bool bown = 15 >= mlo && 15 < mhi;
  int it = 0;
  for (int64_t s = blockIdx.x; s < a.nstrip; s += gridDim.x) {
    const int64_t s0 = s * ST_OWN - ST_HALO;
    const int64_t rb = s0 + 16 * wave;
    // ---- to_params dgrad (1x1, x scale, mask g2) for rows rb - 1 .. rb + 16: two blocks -> dg2, slot
    {
      float4 mA[4], mB[4], xA, xB;
      load_mask(a.g2, rb - 1, R, lg4, l16, mA);
      load_mask(a.g2, rb + 1, R, lg4, l16, mB);
      auto ld_dpar = [&](int64_t r) {  // row r, channels 4 lg4 .. (x_mask: rows outside / pad channels 0)
        const int64_t rc = r < 0 ? 0 : (r >= R ? R - 1 : r);
        const float4 v = *reinterpret_cast<const float4*>(a.dpar + rc * a.ldp + min(4 * lg4, a.ldp - 4));
        return (r >= 0 && r < R && 4 * lg4 < a.ldp) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      };
      xA = ld_dpar(rb - 1 + l16);
      xB = ld_dpar(rb + 1 + l16);
      f32x4 acc[4], acc2[4];
      const float bA[4] = {xA.x, xA.y, xA.z, xA.w}, bB[4] = {xB.x, xB.y, xB.z, xB.w};
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc2[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          acc[nb] = mfma16x16x4(wP[nb][e], bA[e], acc[nb]);
          acc2[nb] = mfma16x16x4(wP[nb][e], bB[e], acc2[nb]);
        }
      mask_epi(acc, mA, psc, rb - 1, R, T, lg4, l16, alo, ahi, a.dg2, slot, ST_LDW);
      mask_epi(acc2, mB, psc, rb + 1, R, T, lg4, l16, bown ? 14 : 16, bown ? 15 : 16, a.dg2, slot + 2 * ST_LDW,
               ST_LDW);
    }
    float4 m1[4];
    load_mask(a.g1, rb, R, lg4, l16, m1);
    if (it == 0) {  // the first strip: every wave's share of the image DMA has landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    } else {
      __builtin_amdgcn_wave_barrier();
    }
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
    const char* e = getenv("VQHMM_STRIP_DBG");
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

int launch_strip_fwd(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2, hipStream_t s) {
  if (!strip_fwd_supported(e1, e2, d1, d2)) return VQHMM_EUNSUPPORTED;
  const StripFwdArgs a = strip_fwd_args(e1, e2, d1, d2);
  const unsigned grid = (unsigned)(a.nstrip < 256 ? a.nstrip : 256);
#define VQHMM_SF(NB2, P) strip_fwd_kernel<NB2, P><<<grid, 512, sizeof(StripFwdLds<NB2>), s>>>(a)
  const bool prof = prof_on() != 0;
  if (c2_nb(e2.N) == 1) {
    if (prof) VQHMM_SF(1, 1); else VQHMM_SF(1, 0);
  } else {
    if (prof) VQHMM_SF(2, 1); else VQHMM_SF(2, 0);
  }
#undef VQHMM_SF
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm

