// Backward strip with the six weight gradients folded in (loss.backward() of VQ_VAE_HMM_fixed.py:156 through
// Encoder.forward :38-41 and Decoder.forward :80-90): the data-gradient chain of strip.hip's strip_bwd_kernel
// (to_params dgrad -> dec_conv2 dgrad -> composed dec_conv1 dgrad + softmax backward + to_logits dgrad ->
// enc_conv2 dgrad, the same MFMA sequences and epilogue arithmetic, so the same bits) and, beside it, every
// layer's weight and bias gradient over the strip's owned rows, accumulated in registers across the
// workgroup's strips and written once per workgroup as a slab row.  The output gradients dY never leave the
// chip and the separate weight-gradient launch (wgrad2_group_kernel: its own fixed costs, a second HBM read
// of every dY and X) is gone.
//
// dW[o][c][tap] = sum_r dY[r][o] X[r + tap - 1][c] over owned rows r: dY of every layer is exact on the owned
// rows (the chain's inexact halo rows are the window's outer two), and X comes from HBM (exact anywhere).
// One MFMA per 16 x 16 tile per 4 rows (K = rows); the 86 tiles of the six layers are split over the 8 waves
// (11 / 10 per wave, 44 accumulator registers), so each wave runs its tiles over ALL owned rows and every
// operand is read from a window-wide LDS buffer: dY where the chain already keeps it (dg2 in the slots, dg1,
// dh2), X staged from the mask registers or HBM.  LDS is time-multiplexed per strip (the dgrad images are
// streamed in per strip by DMA; at the strong-scaling shard sizes a workgroup runs one or two strips):
//
//   region  P1..P2          P3..P4                P5..P6            P7..P8
//   RW      dec_conv2 image G2 | DP | DL          H1 | DL           (next strip's image, DMA)
//   RS      slots (dg2)     D1 (dg1)              H2                DH1
//   RG      G1              enc_conv2 image (DMA, used in P6)
//   RD      -               Dh2 (P4 ->)           Dh2               XX
//   RC      composed dec_conv1 image (output rows 0..3), all strips
//   RE      Q (P1 -> P4)
//
//   P1 front (1x1 to_params dgrad) -> slots; G1 <- g1 mask; Q <- q     P2 dec_conv2 dgrad; W dec_conv2
//   P3 D1 <- dg1; G2 <- g2 mask; DP <- dpar; enc_conv2 image DMA       P4 dec_conv1 dgrad (+ dlog -> DL, dh2 -> Dh2);
//                                                                         W to_params (waves 0-3), dec_conv1' (4-7)
//   P5 H1 <- h1e mask; H2 <- h2e                                      P6 enc_conv2 dgrad; W enc_conv2, to_logits (0-1)
//   P7 DH1 <- dh1; XX <- x; next image DMA                            P8 W enc_conv1 (waves 4-7)
#include "vqhmm.h"

#include <stddef.h>

#include "prof.h"
#include "strip_dev.h"

namespace vqhmm {

__device__ float g_bwdw_one = 1.0f;  // the scale behind a null scale pointer

namespace {
constexpr int SW_LDD = 24;  // dpar rows in LDS (ldp <= 16 channels; 2 * 24 = 16 mod 32: conflict-free column reads)
constexpr int SW_LDQ = 8;   // q / x / dlog rows in LDS

struct StripWLds {
  float RW[3 * 64 * ST_LDW];        // 13824
  float RS[8 * 18 * ST_LDW];        // 10368
  float RG[ST_WIN * ST_LDW];        // 9216
  float RD[(ST_WIN + 2) * SB_LDE];  // 5200
  float RC[4 * 256];                // 3 * 4 * ST_LDW = 864 used; padded to four whole 1-KB DMA chunks
  float RE[ST_WIN * SW_LDQ];        // 1024
  float TW[4 * 32];                 // to_logits' weight (K <= 4, H2 <= 32), zero-padded
};
constexpr int RW_DP = ST_WIN * ST_LDW;           // DP after G2
constexpr int RW_DL = RW_DP + ST_WIN * SW_LDD;   // DL after DP
static_assert(RW_DL + ST_WIN * SW_LDQ <= 3 * 64 * ST_LDW, "G2 | DP | DL fit the dec_conv2 image region");
static_assert(3 * 64 * SB_LDE <= ST_WIN * ST_LDW, "the enc_conv2 image fits the G1 region");
static_assert((ST_WIN + 2) * ST_LDW <= 8 * 18 * ST_LDW && ST_WIN * SB_LDE <= 8 * 18 * ST_LDW,
              "D1 / H2 / DH1 fit the slots region");
static_assert(sizeof(StripWLds) <= 163840, "LDS");

struct SWArgs {
  int64_t R;
  int T, ldp, D, K, H2, own;
  const float* dpar;
  const float *g2, *g1, *h1e, *q, *h2e, *xp;
  const float *img_pd, *img_d2, *img_c1, *img_e2;
  const float* gscale;
  float *dg2, *dg1, *dh1;  // only with store
  int store;
  const float* cmpW;
  float* slab[6];
  float* bslab[6];
  float* cslab;
  int64_t* step_inc;
  int64_t nstrip;
  int prof_it;  // profiling build: the strip index (per workgroup) whose phases are stamped
};

// c2_mfma_tile<1, 1, 4, 3, ST_LDW, 16>'s pipelined sequence on a compact image holding only output rows
// n < 4 of each tap (the full image's rows n >= 4 are zero: lanes l16 >= 4 use 0, the same bits)
__device__ __forceinline__ void c2_tile_n4(const float* Wc, const float* Xw, int lg4, int l16, f32x4& acc) {
  constexpr int KCP = 4, NSTEP = 3 * KCP;
  const bool live = l16 < 4;
  const int wrow = live ? l16 : 0;
  float4 av[2], bv[2];
  auto load = [&](int st, float4& a, float4& b) __attribute__((always_inline)) {
    const int tap = st / KCP, kk = st - tap * KCP;
    const int col = kk * 16 + 4 * lg4;
    const float4 w = *reinterpret_cast<const float4*>(Wc + (tap * 4 + wrow) * ST_LDW + col);
    a = live ? w : make_float4(0.f, 0.f, 0.f, 0.f);
    b = *reinterpret_cast<const float4*>(Xw + (l16 + tap) * ST_LDW + col);
  };
  load(0, av[0], bv[0]);
#pragma unroll
  for (int st = 0; st < NSTEP; ++st) {
    const int cb = st & 1;
    if (st + 1 < NSTEP) load(st + 1, av[cb ^ 1], bv[cb ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
    acc = mfma16x16x4(av[cb].x, bv[cb].x, acc);
    acc = mfma16x16x4(av[cb].y, bv[cb].y, acc);
    acc = mfma16x16x4(av[cb].z, bv[cb].z, acc);
    acc = mfma16x16x4(av[cb].w, bv[cb].w, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One wave's tiles of a weight gradient over the owned window rows [lo, lo + 4 nstep): per 4-row step one
// MFMA per tile, lane group lg4 taking row lo + 4 k + rm; A = fa(row) (dY[row][o] of this lane's output
// channel), B of tile t = fb(row, t) (X[row + tap - 1][c]); bacc += A (the bias gradient's partial).  The
// next step's operands are read while this step's MFMAs run (two register sets, unrolled by two; the
// read past the last step is clamped to it).
template <int NT, class FA, class FB>
__device__ __forceinline__ void wg_pass(int lo, int nstep, int rm, FA fa, FB fb, f32x4 (&acc)[NT], float& bacc) {
  float a0, a1, b0[NT], b1[NT];
  auto load = [&](int k, float& av, float (&bv)[NT]) __attribute__((always_inline)) {
    const int row = lo + 4 * k + rm;
    av = fa(row);
#pragma unroll
    for (int t = 0; t < NT; ++t) bv[t] = fb(row, t);
  };
  auto mma = [&](float av, const float (&bv)[NT]) __attribute__((always_inline)) {
    bacc += av;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(av, bv[t], acc[t]);
  };
  if constexpr (NT == 1) {
    // one 32-cycle MFMA per step cannot hide an LDS read one step ahead: a ring of four operand sets
    // (three steps' reads in flight), the same k order (so the same sums)
    float ar[4], br[4][1];
#pragma unroll
    for (int j = 0; j < 4; ++j) load(min(j, nstep - 1), ar[j], br[j]);
    int k = 0;
    for (; k + 4 <= nstep; k += 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __builtin_amdgcn_sched_barrier(0);
        mma(ar[j], br[j]);
        __builtin_amdgcn_sched_barrier(0);
        load(min(k + 4 + j, nstep - 1), ar[j], br[j]);  // reads past the last step are clamped to it (unused)
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (k + j < nstep) mma(ar[j], br[j]);
    (void)a0; (void)a1; (void)b0; (void)b1;
    return;
  }
  load(0, a0, b0);
  int k = 0;
  for (; k + 1 < nstep; k += 2) {
    load(k + 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    load(min(k + 2, nstep - 1), a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (k < nstep) mma(a0, b0);
}

// the lane-group partials of a bias column summed in a fixed order: (g0 + g1) + (g2 + g3) on every lane
__device__ __forceinline__ float col_sum4(float v) {
  v += xor16(v);
  v += xor32(v);
  return v;
}
// dec_conv1's data-gradient epilogue for the folded strip: conv2_epilogue<1, 1, 3>'s arithmetic (the softmax
// backward of q = softmax(logits) and to_logits' masked dgrad) on operands the caller loaded a phase ahead
// (q, dqx, dlx of row r; h2e channels 8 lg4 .. 8 lg4 + 7 of it; to_logits' weight in LDS), writing dh2 to LDS
// row xs_dh (channels 8 lg4 ..) and dl[0..3] to LDS row xs_dl; nothing to HBM
__device__ __forceinline__ void dec1_epi(f32x4 acc, float sc, int64_t r, int64_t R, int T, int lg4, int l16, float lsc,
                                         const f32x4 (&qdl)[3], const f32x4 (&h4)[2], const float* TWs, float* xs_dh,
                                         float* xs_dl) {
  const bool valid = row_valid(r, R, T);
  f32x4 y;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const float yy = acc[v] * sc + 0.f;
    y[v] = valid ? yy : 0.f;
  }
  float yk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) yk[k] = __shfl(y[k], l16);  // channels 0..3 of row l16 sit in lane l16 (lg4 = 0)
  if (r >= 0 && r < R) {
    float dq[4], sdot = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dq[k] = yk[k] + lsc * qdl[1][k];
      sdot = fmaf(qdl[0][k], dq[k], sdot);
    }
    float dl[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) dl[k] = qdl[0][k] * (dq[k] - sdot) + lsc * qdl[2][k];
    if (lg4 == 0) *reinterpret_cast<f32x4*>(xs_dl + l16 * SW_LDQ) = f32x4{dl[0], dl[1], dl[2], dl[3]};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c0 = 8 * lg4 + 4 * j;
      f32x4 o;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float sacc = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) sacc = fmaf(TWs[k * 32 + c0 + v], dl[k], sacc);
        o[v] = h4[j][v] > 0.f ? sacc : 0.f;
      }
      *reinterpret_cast<f32x4*>(xs_dh + l16 * SB_LDE + c0) = o;
    }
  } else {  // rows outside [0, R): the zero padding of the next conv
#pragma unroll
    for (int j = 0; j < 2; ++j) *reinterpret_cast<f32x4*>(xs_dh + l16 * SB_LDE + 8 * lg4 + 4 * j) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (lg4 == 0) *reinterpret_cast<f32x4*>(xs_dl + l16 * SW_LDQ) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}
}  // namespace

template <int PROF>
__global__ __launch_bounds__(512) void strip_bwdw_kernel(SWArgs a, ConvArgs f) {
  extern __shared__ float4 smem4[];
  StripWLds& sh = *reinterpret_cast<StripWLds*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int64_t R = a.R;
  const int T = a.T, own = a.own, nstep = own / 4;
  constexpr int lo = ST_HALO;  // first owned window row
  float* slot = sh.RS + wave * 18 * ST_LDW;
  if (a.step_inc && blockIdx.x == 0 && tid == 0) *a.step_inc = (*a.step_inc & 0xffffffffll) + 1;

  stamp<PROF>(0);
  if constexpr (PROF > 0) { if (tid == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 13] = __builtin_amdgcn_s_memtime(); }
  const int K = a.K, D = a.D;  // packed-tap gathers (k = 3, 3 C <= 16): B column j = l16 -> (tap, c)
  // ---- once: the compact composed dec_conv1 image (rows n < 4 of each tap) by LDS DMA (to_logits' weight goes
  // to LDS in the first strip's P3)
  // to_logits' weight (K, H2) zero-padded to [4][32] (dec1_epi), through registers, its load ahead of the DMA
  float twv = 0.f;
  if (tid < 128) {
    const int k = tid >> 5, c = tid & 31;
    twv = (k < K && c < a.H2) ? f.lb_W[k * a.H2 + c] : 0.f;
  }
  {
    constexpr int NC = 3 * 4 * ST_LDW / 4;  // float4s: tap t's rows 0..3 are 72 float4s at image row 16 t
    static_assert(NC <= 4 * 64 && sizeof(StripWLds::RC) == 4 * 1024, "one whole-chunk DMA per wave");
    // ONE unguarded instruction in every wave (waves 4-7 copy chunk 3 again, lanes past the image its last
    // float4 into RC's padding: the same bytes), so no branch joins and the compiler counts it exactly
    const int c = min(wave, 3);
    const int i = min(c * 64 + lane, NC - 1);
    dma16(a.img_c1 + ((i / 72) * 16 * ST_LDW + (i % 72) * 4), sh.RC + c * 256);
  }
  if (tid < 128) sh.TW[tid] = twv;
  // the dec_conv2 image, 7 DMA instructions in every wave (54 1-KB chunks; waves 6 and 7 copy chunk 53 twice,
  // the same bytes): the first strip waits for its P1 loads with a counted vmcnt that leaves these in flight
  auto dma_d2 = [&]() __attribute__((always_inline)) {
    constexpr int N1 = 3 * 64 * ST_LDW / 4, C1 = N1 / 64;
    static_assert(N1 % 64 == 0 && C1 <= 56, "7 whole chunks per wave");
#pragma unroll
    for (int j = 0; j < 7; ++j) {  // unguarded (no branch join: the compiler counts these exactly)
      const int c = min(wave + 8 * j, C1 - 1);
      dma16(a.img_d2 + 4 * (c * 64 + lane), sh.RW + c * 256);
    }
  };

  f32x4 accD2[6], accE2[3], accS0[1], accS1[1];  // dec_conv2, enc_conv2; waves 0-3 to_params / to_logits,
  float bD2 = 0.f, bE2 = 0.f, bS0 = 0.f, bS1 = 0.f;  // 4-7 dec_conv1' / enc_conv1 (+ bias partials)
#pragma unroll
  for (int t = 0; t < 6; ++t) accD2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 3; ++t) accE2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  accS0[0] = accS1[0] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int mlo = lo - 16 * wave, mhi = lo + own - 16 * wave;
  const int slo = max(0, mlo), shi = min(16, mhi);
  // ---- each layer's partial gradient -> slab row blockIdx.x (tail_kernel sums the rows), after the last strip
  const int64_t ch = blockIdx.x;
  // the two 64-wide layers' rows are stored output-fastest, [(c * 3 + tap) * O + o] (one 16-byte store per
  // accumulator tile row instead of four scattered words; the tail maps the columns back, SlabSeg::trO)
  auto store_d2 = [&](int lg4, int l16) __attribute__((always_inline)) {  // dec_conv2 (64, 64, 3)
    float* out = a.slab[1] + ch * 64 * 64 * 3;
    const int ob = wave >> 1;
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const int c = ((wave & 1) * 2 + t / 3) * 16 + l16;
      *reinterpret_cast<f32x4*>(out + (c * 3 + t % 3) * 64 + ob * 16 + 4 * lg4) = accD2[t];
    }
    const float cb = col_sum4(bD2);
    if ((wave & 1) == 0 && lg4 == 0) a.bslab[1][ch * 64 + ob * 16 + l16] = cb;
  };
  auto store_s0 = [&](int lg4, int l16, int qtap, int qc, bool qok) __attribute__((always_inline)) {
    const float cb = col_sum4(bS0);
    if (wave < 4) {  // to_params (2D, 64)
      const int P = 2 * D;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int o = 4 * lg4 + v;
        if (o < P) a.slab[0][(ch * P + o) * 64 + wave * 16 + l16] = accS0[0][v];
      }
      if (wave == 0 && lg4 == 0 && l16 < P) a.bslab[0][ch * P + l16] = cb;
    } else {  // composed dec_conv1 (64, K, 3)
      const int ob = wave - 4;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (qok) a.slab[2][((ch * 64 + ob * 16 + 4 * lg4 + v) * K + qc) * 3 + qtap] = accS0[0][v];
      if (lg4 == 0) a.bslab[2][ch * 64 + ob * 16 + l16] = cb;
    }
  };
  auto store_e2 = [&](int lg4, int l16) __attribute__((always_inline)) {  // enc_conv2 (H2, 64, 3), to_logits (K, H2)
    const int H2 = a.H2, ob = wave & 1;
    float* out = a.slab[4] + ch * H2 * 64 * 3;
    const int c = (wave >> 1) * 16 + l16, o0 = ob * 16 + 4 * lg4;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float* dst = out + (c * 3 + t) * H2 + o0;
      if (H2 % 4 == 0) {
        if (o0 < H2) *reinterpret_cast<f32x4*>(dst) = accE2[t];
      } else {
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (o0 + v < H2) dst[v] = accE2[t][v];
      }
    }
    const float ce = col_sum4(bE2), cl = col_sum4(bS1);
    if (wave < 2 && lg4 == 0 && ob * 16 + l16 < H2) a.bslab[4][ch * H2 + ob * 16 + l16] = ce;
    if (wave < 2) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int o = 4 * lg4 + v, c = wave * 16 + l16;
        if (o < K && c < H2) a.slab[3][(ch * K + o) * H2 + c] = accS1[0][v];
      }
      if (wave == 0 && lg4 == 0 && l16 < K) a.bslab[3][ch * K + l16] = cl;
    }
  };
  auto store_e1 = [&](int lg4, int l16, int xtap, int xc, bool xok) __attribute__((always_inline)) {  // enc_conv1
    if (wave < 4) return;
    const int ob = wave - 4;
#pragma unroll
    for (int v = 0; v < 4; ++v)
      if (xok) a.slab[5][((ch * 64 + ob * 16 + 4 * lg4 + v) * D + xc) * 3 + xtap] = accS1[0][v];
    const float cb = col_sum4(bS1);
    if (lg4 == 0) a.bslab[5][ch * 64 + ob * 16 + l16] = cb;
  };

  int it = 0;
  for (int64_t s = blockIdx.x; s < a.nstrip; s += gridDim.x) {
    const bool last = s + gridDim.x >= a.nstrip;  // this workgroup's last strip: P7 stages the dE share
    // the lane ids re-derived opaquely per strip: the per-lane addresses below are recomputed here instead of
    // being hoisted out of the loop as 64-bit VGPR pairs (the accumulators need those registers)
    int tidv = tid;
    asm volatile("" : "+v"(tidv));
    if (it == a.prof_it) stamp<PROF>(15);  // the profiled strip's start (VQHMM_STRIP_PROF_IT)
    // the device scalars, per strip (L2-hot after the first), as VECTOR loads (opaque zero index) issued ahead
    // of P1's loads: waited with them.  Loaded once before the loop they cost the first strip a vmcnt(0)
    // (a register copy of the value) that also waited for the compact image's DMA
    // (unconditional: a null pointer selects the device constant 1; a branch per load would join before the DMA)
    const int z0 = tidv >> 10;  // 0 (tidv < 512), opaque to the compiler
    const float psc = (a.gscale ? a.gscale : &g_bwdw_one)[z0];
    const float fsc = (f.scale ? f.scale : &g_bwdw_one)[z0];
    const float lsc = (f.lb_scale ? f.lb_scale : &g_bwdw_one)[z0];
    const int lane = tidv & 63, lg4 = lane >> 4, l16 = lane & 15;
    const int rm = ((lg4 & 1) << 1) | (lg4 >> 1);  // rows 2 apart in each 32-lane half: conflict-free b32 reads
    const int qtap = l16 / K, qc = l16 - qtap * K;
    const bool qok = l16 < 3 * K;
    const int xtap = l16 / D, xc = l16 - xtap * D;
    const bool xok = l16 < 3 * D;
    const int64_t s0 = s * own - ST_HALO;  // PCL row of window row 0
    const int64_t rb = s0 + 16 * wave;
    // dpar row r, channels 4 lg4 ..: the raw load from a clamped address, and its mask (rows outside / pad
    // channels 0) applied where it is used, so no wait sits right behind the load
    auto ld_dpar_raw = [&](int64_t r) {
      const int64_t rc = r < 0 ? 0 : (r >= R ? R - 1 : r);
      return *reinterpret_cast<const float4*>(a.dpar + rc * a.ldp + min(4 * lg4, a.ldp - 4));
    };
    auto dpar_mask = [&](int64_t r, float4 v) {
      return (r >= 0 && r < R && 4 * lg4 < a.ldp) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    // ================= P1: the 1x1 to_params dgrad -> slots (as strip_bwd_kernel); G1 <- g1; Q <- q
    float4 m1[4];
    {
      float wP[4][4];  // A operand of the 1x1 front: image[n = nb*16 + l16][k = 4 lg4 + e] (L2)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float4 w4 = *reinterpret_cast<const float4*>(a.img_pd + (nb * 16 + l16) * ST_LDF + 4 * lg4);
        wP[nb][0] = w4.x; wP[nb][1] = w4.y; wP[nb][2] = w4.z; wP[nb][3] = w4.w;
      }
      load_mask(a.g1, rb, R, lg4, l16, m1);
      auto front = [&](const float4 x, f32x4 (&acc)[4]) {
        const float b[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma16x16x4(wP[nb][e], b[e], acc[nb]);
      };
      const bool extra = wave == 5 || wave == 6;
      const int64_t re = wave == 5 ? s0 - 1 : s0 + 16 * 7 + 1;
      // every load of this phase unconditional (clamped addresses; only the waves that need a value use it):
      // a branch join before the image DMA below would make the compiler drain vmcnt before the front
      float4 mA[4], xA, mB[4], xB;
      load_mask(a.g2, rb, R, lg4, l16, mA);
      xA = ld_dpar_raw(rb + l16);
      load_mask(a.g2, re, R, lg4, l16, mB);  // waves 5 and 6: the window's outer rows
      xB = ld_dpar_raw(re + l16);
      float4 qv;
      {
        int64_t r = s0 + (tidv & (ST_WIN - 1));
        r = r < 0 ? 0 : (r >= R ? R - 1 : r);
        qv = *reinterpret_cast<const float4*>(a.q + r * 4);  // ld4(K) = 4; rows of threads < ST_WIN
      }
      asm volatile("" ::: "memory");
      if (it == a.prof_it) stamp<PROF>(10);
      f32x4 acc[4];
      front(dpar_mask(rb + l16, xA), acc);
      if constexpr (PROF > 0) {
        if (it == a.prof_it) {
          asm volatile("s_nop 0" : : "v"(acc[3][3]));
          stamp<PROF>(11);
        }
      }
      mask_epi(acc, mA, psc, rb, R, T, lg4, l16, slo, shi, a.store ? a.dg2 : nullptr, slot + ST_LDW, ST_LDW, -1,
               wave > 0 ? slot - 18 * ST_LDW + 17 * ST_LDW : nullptr, wave < 7 ? slot + 18 * ST_LDW : nullptr);
      if (extra) {
        f32x4 acc2[4];
        front(dpar_mask(re + l16, xB), acc2);
        mask_epi(acc2, mB, psc, re, R, T, lg4, l16, 0, 0, nullptr,
                 wave == 5 ? sh.RS : sh.RS + 7 * 18 * ST_LDW + 2 * ST_LDW, ST_LDW, wave == 5 ? 0 : 15);
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        *reinterpret_cast<float4*>(sh.RG + (16 * wave + l16) * ST_LDW + nb * 16 + 4 * lg4) = m1[nb];
      if (tidv < ST_WIN) *reinterpret_cast<float4*>(sh.RE + tidv * SW_LDQ) = qv;
    }
    if (it == a.prof_it) stamp<PROF>(12);
    // the dec_conv2 image for P2's dgrad tile (RW is free since B6 of the last strip): issued after P1 consumed
    // its loads, the 7 youngest vmcnt events, in flight through B1 and P2's weight-gradient pass
    dma_d2();
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // (P1's loads: already consumed)
    lds_barrier_dma();  // B1: slots, G1, Q
    if (it == a.prof_it) stamp<PROF>(1);
    // ================= P2: dec_conv2 weight gradient (needs no image: hides the first strip's image DMA), then
    // dec_conv2 dgrad (mask g1) -> dg1 (registers)
    f32x4 mA[4];  // g2 / dpar rows again (L2), for G2 / DP in P3: in flight across this phase
    {
      int64_t r = rb + l16;
      r = r < 0 ? 0 : (r >= R ? R - 1 : r);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) mA[nb] = *reinterpret_cast<const f32x4*>(a.g2 + r * 64 + nb * 16 + 4 * lg4);
    }
    const float4 xA = ld_dpar_raw(rb + l16);  // masked when stored (P3)
    {  // tiles (ob = wave / 2, cb = 2 (wave % 2) + j, tap): dY = dg2 (slots), X = g1 (G1)
      const float* ya = sh.RS + (wave >> 1) * 16 + l16;
      const float* xb = sh.RG + (wave & 1) * 32 + l16;
      wg_pass<6>(lo, nstep, rm,
                 [&](int row) { return ya[(row >> 4) * 18 * ST_LDW + ((row & 15) + 1) * ST_LDW]; },
                 [&](int row, int t) { return xb[(row - 1 + t % 3) * ST_LDW + (t / 3) * 16]; }, accD2, bD2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's share of the image has landed
    lds_barrier_dma();
    f32x4 d1[4];
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<4, 1, 4, 3, ST_LDW, 64>(sh.RW, slot, lg4, l16, acc, true);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) d1[nb] = acc[nb][0];
      mask_epi(d1, m1, 1.0f, rb, R, T, lg4, l16, slo, shi, a.store ? a.dg1 : nullptr, nullptr, 0);
    }
    lds_barrier();  // B2: the slots, G1 and the image are read
    if (it == a.prof_it) stamp<PROF>(2);
    // ================= P3: D1 <- dg1, G2 <- g2, DP <- dpar; the enc_conv2 image by DMA into the G1 region;
    // P4's epilogue operands in flight
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      *reinterpret_cast<f32x4*>(sh.RS + (16 * wave + 1 + l16) * ST_LDW + nb * 16 + 4 * lg4) = d1[nb];
      *reinterpret_cast<f32x4*>(sh.RW + (16 * wave + l16) * ST_LDW + nb * 16 + 4 * lg4) = mA[nb];
    }
    *reinterpret_cast<float4*>(sh.RW + RW_DP + (16 * wave + l16) * SW_LDD + 4 * lg4) = dpar_mask(rb + l16, xA);
    // the enc_conv2 image (30 KB) through registers, stored to RG (free since B2) at the end of P4: an LDS DMA
    // would be drained at P4's first LDS read (the compiler cannot tell its destination from P4's operands)
    constexpr int N2 = 3 * 64 * SB_LDE / 4, C2 = N2 / 64;
    static_assert(N2 % 64 == 0 && C2 <= 32, "4 whole chunks per wave");
    f32x4 e2v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // a fixed count (the last chunk again where a wave has 3: the same bytes)
      const int c = min(wave + 8 * j, C2 - 1);
      e2v[j] = *reinterpret_cast<const f32x4*>(a.img_e2 + 4 * (c * 64 + lane));
    }
    f32x4 qdl[3], h4[2];  // q, dqx, dlx of row rb + l16 and h2e channels 8 lg4 .. + 7 of it (dec1_epi)
    {
      int64_t r = rb + l16;
      r = r < 0 ? 0 : (r >= R ? R - 1 : r);
      qdl[0] = *reinterpret_cast<const f32x4*>(f.lb_q + r * 4);
      qdl[1] = *reinterpret_cast<const f32x4*>(f.lb_dqx + r * 4);
      qdl[2] = *reinterpret_cast<const f32x4*>(f.lb_dlx + r * 4);
#pragma unroll
      for (int j = 0; j < 2; ++j) h4[j] = *reinterpret_cast<const f32x4*>(f.lb_h + r * 32 + 8 * lg4 + 4 * j);
    }
    lds_barrier_dma();  // B3: D1, G2, DP, TW (the enc_conv2 image DMA stays in flight: waited in P5)
    if (it == a.prof_it) stamp<PROF>(3);
    // ================= P4: composed dec_conv1 dgrad + softmax backward + to_logits dgrad (dh2 -> Dh2, dlog -> DL);
    // to_params weight gradient (waves 0-3), composed dec_conv1's (waves 4-7)
    f32x4 h2v[2];  // h2e rows for P5, in flight across this phase
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tidv + 512 * j, row = i >> 3;
      int64_t r = s0 + row;
      r = r < 0 ? 0 : (r >= R ? R - 1 : r);
      h2v[j] = *reinterpret_cast<const f32x4*>(a.h2e + r * 32 + (i & 7) * 4);
    }
    {
      f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_tile_n4(sh.RC, sh.RS + 16 * wave * ST_LDW, lg4, l16, acc1);
      dec1_epi(acc1, fsc, rb + l16, R, T, lg4, l16, lsc, qdl, h4, sh.TW, sh.RD + (16 * wave + 1) * SB_LDE,
               sh.RW + RW_DL + 16 * wave * SW_LDQ);
    }
    if (wave < 4) {  // to_params: tile (0, cb = wave), 1x1: dY = dpar (DP), X = g2 (G2)
      const float* ya = sh.RW + RW_DP + l16;
      const float* xb = sh.RW + wave * 16 + l16;
      wg_pass<1>(lo, nstep, rm, [&](int row) { return ya[row * SW_LDD]; },
                 [&](int row, int) { return xb[row * ST_LDW]; }, accS0, bS0);
    } else {  // composed dec_conv1: tile (ob = wave - 4, packed taps): dY = dg1 (D1), X = q (Q)
      const float* ya = sh.RS + ST_LDW + (wave - 4) * 16 + l16;
      const float* xb = sh.RE + qc;
      wg_pass<1>(lo, nstep, rm, [&](int row) { return ya[row * ST_LDW]; },
                 [&](int row, int) { const float v = xb[(row - 1 + (qok ? qtap : 0)) * SW_LDQ]; return qok ? v : 0.f; },
                 accS0, bS0);
    }
    float4 m2[4];  // h1e rows: H1 in P5, enc_conv2 dgrad's mask in P6
    load_mask(a.h1e, rb, R, lg4, l16, m2);
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(sh.RG + min(wave + 8 * j, C2 - 1) * 256 + 4 * lane) = e2v[j];
    lds_barrier_dma();  // B4: D1, G2, DP, Q are read; Dh2, DL and the enc_conv2 image written
    if (it == a.prof_it) stamp<PROF>(4);
    // ================= P5: H1 <- h1e (RW, beside DL), H2 <- h2e (RS)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      *reinterpret_cast<float4*>(sh.RW + (16 * wave + l16) * ST_LDW + nb * 16 + 4 * lg4) = m2[nb];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tidv + 512 * j;
      *reinterpret_cast<f32x4*>(sh.RS + (i >> 3) * SB_LDE + (i & 7) * 4) = h2v[j];
    }
    lds_barrier();  // B5
    if (it == a.prof_it) stamp<PROF>(5);
    // ================= P6: enc_conv2 dgrad (mask h1) -> dh1 (registers); the enc_conv2 and to_logits (waves 0-1)
    // weight gradients
    const int xsh = ld4(D) == 8 ? 1 : 0;
    float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);  // x rows for P7: thread = (row, float4 of the ld4(D) <= 8 row)
    if (tidv < (ST_WIN << xsh)) {
      int64_t r = s0 + (tidv >> xsh);
      r = r < 0 ? 0 : (r >= R ? R - 1 : r);
      xv = *reinterpret_cast<const float4*>(a.xp + (r << (2 + xsh)) + (tidv & xsh) * 4);
    }
    f32x4 y[4];
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<4, 1, 2, 3, SB_LDE, 64>(sh.RG, sh.RD + 16 * wave * SB_LDE, lg4, l16, acc, true);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) y[nb] = acc[nb][0];
      mask_epi(y, m2, 1.0f, rb, R, T, lg4, l16, slo, shi, a.store ? a.dh1 : nullptr, nullptr, 0);
    }
    {  // tiles (ob = wave % 2, cb = wave / 2, tap): dY = dh2 (Dh2), X = h1e (H1)
      const float* ya = sh.RD + SB_LDE + (wave & 1) * 16 + l16;
      const float* xb = sh.RW + (wave >> 1) * 16 + l16;
      wg_pass<3>(lo, nstep, rm, [&](int row) { return ya[row * SB_LDE]; },
                 [&](int row, int t) { return xb[(row - 1 + t) * ST_LDW]; }, accE2, bE2);
    }
    if (wave < 2) {  // to_logits: tile (0, cb = wave), 1x1: dY = dlog (DL, channels < K), X = h2e (H2)
      const float* ya = sh.RW + RW_DL + min(l16, 3);
      const float* xb = sh.RS + wave * 16 + l16;
      const bool ok = l16 < K;
      wg_pass<1>(lo, nstep, rm, [&](int row) { const float v = ya[row * SW_LDQ]; return ok ? v : 0.f; },
                 [&](int row, int) { return xb[row * SB_LDE]; }, accS1, bS1);
    }
    lds_barrier();  // B6: H1, H2, DL, Dh2 and the enc_conv2 image are read
    if (it == a.prof_it) stamp<PROF>(6);
    // ================= P7: DH1 <- dh1 (RS), XX <- x (RD); the next strip's dec_conv2 image (RW)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      *reinterpret_cast<f32x4*>(sh.RS + (16 * wave + l16) * ST_LDW + nb * 16 + 4 * lg4) = y[nb];
    if (tidv < (ST_WIN << xsh)) *reinterpret_cast<float4*>(sh.RD + (tidv >> xsh) * SW_LDQ + (tidv & xsh) * 4) = xv;
    if (last) {  // after the loop: decoder.conv1's weight (64, 64, 3) for the dE share (LDS DMA, 48 chunks of 1 KB),
      // the share's dWc buffer zeroed (RG: the enc_conv2 image is read)
#pragma unroll
      for (int j = 0; j < 6; ++j) dma16(a.cmpW + 4 * ((wave + 8 * j) * 64 + lane), sh.RW + (wave + 8 * j) * 256);
      for (int i = tidv; i < 1536; i += 512) sh.RG[i] = 0.f;
    }
    lds_barrier_dma();  // B7 (the next strip's image DMA stays in flight: waited before B1)
    // ================= P8: enc_conv1 weight gradient (waves 4-7): tile (ob = wave - 4, packed taps): dY = dh1
    // (DH1), X = x (XX)
    if (wave >= 4) {
      const float* ya = sh.RS + (wave - 4) * 16 + l16;
      const float* xb = sh.RD + xc;
      wg_pass<1>(lo, nstep, rm, [&](int row) { return ya[row * ST_LDW]; },
                 [&](int row, int) { const float v = xb[(row - 1 + (xok ? xtap : 0)) * SW_LDQ]; return xok ? v : 0.f; },
                 accS1, bS1);
    }
    lds_barrier_dma();  // B8: DH1 and XX are read before the next strip writes the slots
    if (it == a.prof_it) stamp<PROF>(7);
    ++it;
  }

  {
    const int qtap = l16 / K, qc = l16 - qtap * K;
    const bool qok = l16 < 3 * K;
    const int xtap = l16 / D, xc = l16 - xtap * D;
    const bool xok = l16 < 3 * D;
    store_d2(lg4, l16);
    store_s0(lg4, l16, qtap, qc, qok);
    store_e2(lg4, l16);
    store_e1(lg4, l16, xtap, xc, xok);
  }
  // ---- the composed decoder conv1's embedding-gradient share of this workgroup (wgrad2.hip's
  // wgrad_compose_de over 8 thread groups): cslab[ch][k][h] = sum_{o, tap} dWc[o][k][tap] W[o][h][tap]
  {
    const int qtap = l16 / K, qc = l16 - qtap * K;
    const bool qok = l16 < 3 * K;
    const int h = tid & 63, g = tid >> 6;
    float* cbuf = sh.RG;          // [(o * 3 + tap) * 8 + k], zero for k >= K (zeroed in the last strip's P7)
    float* part = sh.RG + 1536;   // [8 groups][8 k][64 h]
    const float* Wl = sh.RW;      // decoder.conv1's weight (64, 64, 3), DMA'd in the last strip's P7
    if (wave >= 4) {
      const int ob = wave - 4;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (qok) cbuf[((ob * 16 + 4 * lg4 + v) * 3 + qtap) * 8 + qc] = accS0[0][v];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the weight DMA
    lds_barrier();
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int tap = 0; tap < 3; ++tap) {
        const float4* c4 = reinterpret_cast<const float4*>(cbuf + ((g + 8 * i) * 3 + tap) * 8);
        const float4 l = c4[0], hh = c4[1];
        const float cv[8] = {l.x, l.y, l.z, l.w, hh.x, hh.y, hh.z, hh.w};
        const float wv = Wl[((g + 8 * i) * 64 + h) * 3 + tap];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(cv[k], wv, acc[k]);
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) part[(g * 8 + k) * 64 + h] = acc[k];
    lds_barrier();
    if (tid < K * 64) {
      const int k = tid >> 6;
      float v = 0.f;
#pragma unroll
      for (int gg = 0; gg < 8; ++gg) v += part[(gg * 8 + k) * 64 + h];
      a.cslab[ch * K * 64 + tid] = v;
    }
  }
  if constexpr (PROF > 0) {
    __syncthreads();
    stamp<PROF>(8);
    if (threadIdx.x == 0 && blockIdx.x < 256) {
      g_prof[blockIdx.x * 16 + 14] = __builtin_amdgcn_s_memtime();
      g_prof[blockIdx.x * 16 + 9] = (unsigned long long)it;
    }
  }
}

int bwdw_prof_copy(uint64_t* out, int64_t n) { return prof_copy(out, n); }

static int prof_on() {
  static const int v = prof_env("VQHMM_STRIP_PROF");
  return v;
}

bool strip_bwdw_supported(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2, int D) {
  return strip_bwd_supported(pd, d2, f, e2) && D >= 1 && 3 * D <= 16 && pd.Kc == 2 * D && f.N >= 1 && f.N <= 4 &&
         3 * f.N <= 16;
}

// owned rows per strip: a multiple of 4 (the MFMA steps), at most ST_OWN, sized so that the strips cover the
// rows in as few rounds of 256 workgroups as ST_OWN allows with every workgroup busy in the last one
int strip_bwdw_own(int64_t R) {
  const int64_t rounds = cdiv(R, 256ll * ST_OWN);
  const int64_t own = cdiv(cdiv(R, 256 * rounds), 4) * 4;
  return (int)(own < 4 ? 4 : own > ST_OWN ? ST_OWN : own);
}

int strip_bwdw_grid(int64_t R) {
  const int64_t n = cdiv(R, strip_bwdw_own(R));
  return (int)(n < 256 ? (n > 0 ? n : 1) : 256);
}

int launch_strip_bwdw(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2,
                      const StripWgradArgs& w, hipStream_t s) {
  if (!strip_bwdw_supported(pd, d2, f, e2, w.D) || w.H2 != f.lb_C || w.K != f.N) return VQHMM_EUNSUPPORTED;
  SWArgs a{};
  a.R = pd.R; a.T = pd.T; a.ldp = ld4(pd.Kc); a.D = w.D; a.K = w.K; a.H2 = w.H2;
  a.own = strip_bwdw_own(pd.R);
  a.dpar = pd.src; a.g2 = pd.aux; a.g1 = d2.aux; a.h1e = e2.aux; a.q = f.lb_q; a.h2e = f.lb_h; a.xp = w.x;
  a.img_pd = pd.Wimg; a.img_d2 = d2.Wimg; a.img_c1 = f.Wimg; a.img_e2 = e2.Wimg;
  a.gscale = pd.scale;
  a.store = w.store;
  a.dg2 = pd.out; a.dg1 = d2.out; a.dh1 = e2.out;
  a.cmpW = w.cmpW;
  for (int i = 0; i < 6; ++i) {
    a.slab[i] = w.slab[i];
    a.bslab[i] = w.bslab[i];
  }
  a.cslab = w.cslab;
  a.step_inc = w.step_inc;
  a.nstrip = cdiv(pd.R, a.own);
  {
    static const int pit = prof_env("VQHMM_STRIP_PROF_IT");
    a.prof_it = pit;
  }
  const unsigned grid = (unsigned)strip_bwdw_grid(pd.R);
  if (prof_on()) strip_bwdw_kernel<1><<<grid, 512, sizeof(StripWLds), s>>>(a, f);
  else strip_bwdw_kernel<0><<<grid, 512, sizeof(StripWLds), s>>>(a, f);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
