// Wide convolutions (k = 1 or 3, more than 64 channels on a side; Kc a multiple of 16) as an implicit GEMM on
// the f32 MFMA: the cfg3-dims layers (H = 256, H2 = 128, K = 32, D = 64) of VQ_VAE_HMM_fixed.py:34-36,77-79 and
// their data gradients, the 1x1 tails to_logits / to_params (:36, :79) as their own launches, and the staged
// head's Prior MLP layers (:53-57) at K^2 = 1024 transition logits.
//
// GEMM view over PCL rows (common.h): Y[r][n] = sum_{tap, c} X[r + tap - 1][c] Weff[n][c][tap], Weff = W (forward)
// or W[c][n][2 - tap] (data gradient).  A workgroup owns a BM = 128 row x BN column tile; its 4 waves split it
// 2 x 2 (64 rows x BN / 2 columns each: 4 x BN / 32 accumulators of v_mfma_f32_16x16x4_f32).  The reduction
// walks 16-channel slices: the slice's 130 input rows and its 3 x BN weight rows are staged in LDS (rows of 24
// floats: the float4 operand reads of all four 16-lane groups are bank-conflict free), while the next slice's
// operands are already in flight in registers.  Inside a slice lane group g holds channels 4g .. 4g + 3 of its
// row as one float4 and MFMA e uses element e, for A and B alike, so every channel is summed exactly once
// (the k order inside a slice is a fixed permutation; the result is a k-ordered fmaf chain as any f32 MFMA).
//
// Epilogue: scale, bias, ReLU or the ReLU-backward mask (act 2: aux > 0), pad rows zero, PCL store; SOFTMAX
// (N <= BN / 2 <= 64, the tail to_logits): q = softmax over the row's N channels to q_out, through LDS.
#include <algorithm>

#include "kernels.h"

namespace vqhmm {

namespace {
constexpr int CB_BM = 128;  // rows per tile
constexpr int CB_KC = 16;   // channels per slice
constexpr int CB_LD = 24;   // LDS row stride (floats) of the staged X rows and weight rows
}  // namespace

template <int BN>
struct ConvBigCfg {
  static constexpr int WN = BN / 32;                   // 16-col accumulator blocks per wave (2 waves across)
  static constexpr int X4 = (CB_BM + 2) * 4;           // float4s of one slice's X rows
  static constexpr int W4 = 3 * BN * 4;                // float4s of one slice's weight rows (3 taps)
  static constexpr int PX = (X4 + 255) / 256, PW = (W4 + 255) / 256;
  static constexpr int LDS_FLOATS = (CB_BM + 2) * CB_LD + 3 * BN * CB_LD;
};

// One float4 of the slice's weights: source address (or null: zeros) and the 4 LDS destinations (tap, n, c) it
// scatters to.  Forward: per n the slice's (c, tap) pairs are 48 (k = 3) / 16 (k = 1) contiguous floats of W[n];
// data gradient: per c the tile's (n, tap) pairs are 3 BN / BN contiguous floats of W[c].
template <int BN, int LD = CB_LD>
__device__ __forceinline__ const float* cb_wsrc(const ConvArgs& a, int n0, int c0, int q, int (&dst)[4]) {
  const int ks = a.ks;
  if (!a.w_dgrad) {
    const int per_n = 4 * ks;  // float4s per n row of the slice
    const int n = q / per_n, f = q - n * per_n;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = 4 * f + e, c = ks == 3 ? idx / 3 : idx, tap = ks == 3 ? idx - 3 * (idx / 3) : 0;
      dst[e] = (tap * BN + n) * LD + c;
    }
    if (n >= BN || n0 + n >= a.N) return nullptr;
    return a.W + ((int64_t)(n0 + n) * a.Kc + c0) * ks + 4 * f;
  }
  const int per_c = ks * BN / 4;
  const int c = q / per_c, f = q - c * per_c;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = 4 * f + e, n = ks == 3 ? idx / 3 : idx, t = ks == 3 ? idx - 3 * (idx / 3) : 0;
    dst[e] = ((ks - 1 - t) * BN + n) * LD + c;
  }
  if (c >= CB_KC || n0 + (ks == 3 ? (4 * f) / 3 : 4 * f) >= a.N) return nullptr;  // N % 4 == 0: whole float4s
  return a.W + ((int64_t)(c0 + c) * a.N + n0) * ks + 4 * f;
}

// 1-D grid -> (row block, column tile) with the column tiles of one row block back to back on one XCD
// (workgroups are dealt to the 8 XCDs round robin): a row block's X rows then come from that XCD's L2 after the
// first tile instead of from HBM once per column tile.  False for the padding workgroups.
__device__ __forceinline__ bool cb_tile(int64_t nrb, int ny, int64_t& rb, int& ct) {
  const int64_t w = blockIdx.x, xcd = w % 8, k = w / 8;
  ct = (int)(k % ny);
  rb = (k / ny) * 8 + xcd;
  return rb < nrb;
}

// Epilogue shared by the k = 3 / k = 1 kernels: lane (lg, l16), register v -> row wm*64 + i*16 + 4 lg + v,
// column wn*BN/2 + j*16 + l16; Xs is reused as the SOFTMAX staging buffer.
template <int BN, bool SOFTMAX>
__device__ __forceinline__ void cb_epilogue(const ConvArgs& a, f32x4 (&acc)[4][BN / 32], float* Xs, int64_t m0, int n0) {
  constexpr int WN = BN / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg = lane >> 4, l16 = lane & 15;
  const int wm = wave & 1, wn = wave >> 1;
  const float sc = a.scale ? *a.scale : 1.f;
  const int ldn = a.N;  // N % 4 == 0: no pad channels
  // bias and each 16-row block's ReLU-mask operands are loaded before any of its stores: loads after a store to
  // `out` (which may alias them as far as the compiler knows) were each issued and waited for alone
  // (vmcnt(0) 130 times per epilogue)
  float bj[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + l16;
    bj[j] = a.bias && n < a.N ? a.bias[n] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float ax[4][WN];
    if (a.act == 2) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t r = m0 + wm * 64 + i * 16 + 4 * lg + v;
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const int n = n0 + wn * (BN / 2) + j * 16 + l16;
          ax[v][j] = r < a.R && n < a.N ? a.aux[r * ldn + n] : 0.f;
        }
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = wm * 64 + i * 16 + 4 * lg + v;
      const int64_t r = m0 + row;
      int64_t b;
      int t;
      const bool valid = row_bt_fast(r, a.R, a.T, b, t);
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int n = n0 + wn * (BN / 2) + j * 16 + l16;
        float y = acc[i][j][v] * sc;
        if (a.bias && n < a.N) y += bj[j];
        if (a.act == 1) y = relu_f(y);
        else if (a.act == 2 && r < a.R && n < a.N) y = ax[v][j] > 0.f ? y : 0.f;
        y = valid ? y : 0.f;
        acc[i][j][v] = y;
        if (a.out && r < a.R && n < a.N) a.out[r * ldn + n] = y;
      }
    }
  }
  if constexpr (SOFTMAX) {  // q = softmax over the row's N <= BN / 2 channels (all in the wn = 0 waves)
    __syncthreads();
    float* Ys = Xs;  // [BM][BN / 2 + 1]
    constexpr int LY = BN / 2 + 1;
    if (wn == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
          for (int j = 0; j < WN; ++j) Ys[(wm * 64 + i * 16 + 4 * lg + v) * LY + j * 16 + l16] = acc[i][j][v];
    }
    __syncthreads();
    if (tid < CB_BM) {  // thread per row, q written back over the row in LDS
      const int64_t r = m0 + tid;
      int64_t b;
      int t;
      const bool valid = row_bt_fast(r, a.R, a.T, b, t);
      float* y = Ys + tid * LY;
      float mx = -__builtin_inff();
      for (int n = 0; n < a.N; ++n) mx = fmaxf(mx, y[n]);
      float se = 0.f;
      for (int n = 0; n < a.N; ++n) se += __expf(y[n] - mx);
      for (int n = 0; n < a.N; ++n) y[n] = valid ? __expf(y[n] - mx) / se : 0.f;
    }
    __syncthreads();
    // the tile's q rows are one contiguous block of BM x N floats: stored by every thread, consecutive threads
    // on consecutive floats (the thread-per-row stores were 128 B apart per lane)
    const int64_t nq = std::min<int64_t>(CB_BM, a.R - m0) * a.N;
    for (int e = tid; e < nq; e += 256) {
      const int row = e / a.N, n = e - row * a.N;
      a.q_out[m0 * ldn + e] = Ys[row * LY + n];
    }
  }
}

template <int BN, bool SOFTMAX>
__global__ __launch_bounds__(256) void convbig_kernel(ConvArgs a) {
  using C = ConvBigCfg<BN>;
  constexpr int WN = C::WN;
  extern __shared__ float4 smem4[];
  float* Xs = reinterpret_cast<float*>(smem4);  // [(BM + 2)][LD]
  float* Ws = Xs + (CB_BM + 2) * CB_LD;         // [3][BN][LD]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg = lane >> 4, l16 = lane & 15;
  const int wm = wave & 1, wn = wave >> 1;
  int64_t rb;
  int ct;
  if (!cb_tile(cdiv(a.R, CB_BM), (int)cdiv(a.N, BN), rb, ct)) return;
  const int64_t m0 = rb * CB_BM;
  const int n0 = ct * BN;
  const int ldx = a.Kc, ks = a.ks, nslice = a.Kc / CB_KC;
  const int wrows = ks * BN * 4;  // valid weight float4s per slice

  float4 px[C::PX], pw[C::PW];
  auto load = [&](int c0) {
#pragma unroll
    for (int k = 0; k < C::PX; ++k) {
      const int i = tid + 256 * k, row = i >> 2, c4 = (i & 3) * 4;
      const int64_t r = m0 - 1 + row;
      const bool ok = i < C::X4 && r >= 0 && r < a.R;
      px[k] = ok ? *reinterpret_cast<const float4*>(a.src + r * ldx + c0 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < C::PW; ++k) {
      const int q = tid + 256 * k;
      int dst[4];
      const float* src = q < wrows ? cb_wsrc<BN>(a, n0, c0, q, dst) : nullptr;
      pw[k] = src ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int c0) {
#pragma unroll
    for (int k = 0; k < C::PX; ++k) {
      const int i = tid + 256 * k;
      if (i < C::X4) *reinterpret_cast<float4*>(Xs + (i >> 2) * CB_LD + (i & 3) * 4) = px[k];
    }
#pragma unroll
    for (int k = 0; k < C::PW; ++k) {
      int q = tid + 256 * k;
      if (q < wrows) {
        // q made opaque: the 4 LDS destinations are recomputed here, not hoisted out of the slice loop (kept live
        // they cost 4 VGPRs per prefetched float4, a second wave per SIMD)
        asm volatile("" : "+v"(q));
        int dst[4];
        (void)cb_wsrc<BN>(a, n0, c0, q, dst);
        Ws[dst[0]] = pw[k].x;
        Ws[dst[1]] = pw[k].y;
        Ws[dst[2]] = pw[k].z;
        Ws[dst[3]] = pw[k].w;
      }
    }
  };

  f32x4 acc[4][WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  for (int s = 0; s < nslice; ++s) {
    __syncthreads();  // every wave is done reading the previous slice
    store(s * CB_KC);
    __syncthreads();
    if (s + 1 < nslice) load((s + 1) * CB_KC);  // in flight across this slice's MFMAs
    for (int tap = 0; tap < ks; ++tap) {
      const int roff = ks == 3 ? tap : 1;
      float4 av[4], bv[WN];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        av[i] = *reinterpret_cast<const float4*>(Xs + (wm * 64 + i * 16 + l16 + roff) * CB_LD + 4 * lg);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        bv[j] = *reinterpret_cast<const float4*>(Ws + (tap * BN + wn * (BN / 2) + j * 16 + l16) * CB_LD + 4 * lg);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            const float ae = e == 0 ? av[i].x : e == 1 ? av[i].y : e == 2 ? av[i].z : av[i].w;
            const float be = e == 0 ? bv[j].x : e == 1 ? bv[j].y : e == 2 ? bv[j].z : bv[j].w;
            acc[i][j] = mfma16x16x4(ae, be, acc[i][j]);
          }
    }
  }

  cb_epilogue<BN, SOFTMAX>(a, acc, Xs, m0, n0);
}

// k = 1 with Kc % 32 == 0: two 16-channel slices per LDS stage, no halo rows.  One slice per stage left a k = 1
// workgroup 64 MFMAs per wave between a slice's loads and their use, under the load latency: the Prior MLP's
// 1x1 layers (K^2 = 1024 logits and their data gradient) and the 1x1 data gradients ran at 0.21-0.37 of the
// MFMA peak at cfg3.  Same slices in the same order as convbig_kernel: the same fmaf chain, bit for bit.
template <int BN>
struct ConvBig1Cfg {
  static constexpr int SPS = 2;                         // slices per stage
  static constexpr int X4 = CB_BM * 4, W4 = BN * 4;     // float4s of one slice's X rows / weight rows
  static constexpr int PX = X4 / 256, PW = (W4 + 255) / 256;
  // LDS row stride 20 floats: the 16 rows a 16-lane group reads as float4s start at 16 distinct multiples of 4
  // banks (20 r mod 64), all 64 banks once; 40 KB per workgroup at BN = 128, four workgroups per CU
  static constexpr int LD = 20;
  static constexpr int XS = CB_BM * LD, WS = BN * LD;
  static constexpr int LDS_FLOATS = SPS * (XS + WS);
};

template <int BN, bool SOFTMAX>
__global__ __launch_bounds__(256) void convbig1_kernel(ConvArgs a) {
  using C = ConvBig1Cfg<BN>;
  constexpr int WN = BN / 32, SPS = C::SPS;
  extern __shared__ float4 smem4[];
  float* Xs = reinterpret_cast<float*>(smem4);  // [SPS][BM][LD]
  float* Ws = Xs + SPS * C::XS;                 // [SPS][BN][LD]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg = lane >> 4, l16 = lane & 15;
  const int wm = wave & 1, wn = wave >> 1;
  int64_t rb;
  int ct;
  if (!cb_tile(cdiv(a.R, CB_BM), (int)cdiv(a.N, BN), rb, ct)) return;
  const int64_t m0 = rb * CB_BM;
  const int n0 = ct * BN;
  const int ldx = a.Kc, nstage = a.Kc / (CB_KC * SPS);

  float4 px[SPS][C::PX], pw[SPS][C::PW];
  auto load = [&](int c0) {
#pragma unroll
    for (int h = 0; h < SPS; ++h) {
#pragma unroll
      for (int k = 0; k < C::PX; ++k) {
        const int i = tid + 256 * k, row = i >> 2, c4 = (i & 3) * 4;
        const int64_t r = m0 + row;
        px[h][k] = r < a.R ? *reinterpret_cast<const float4*>(a.src + r * ldx + c0 + CB_KC * h + c4)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < C::PW; ++k) {
        const int q = tid + 256 * k;
        int dst[4];
        const float* src = q < C::W4 ? cb_wsrc<BN, C::LD>(a, n0, c0 + CB_KC * h, q, dst) : nullptr;
        pw[h][k] = src ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int h = 0; h < SPS; ++h) {
#pragma unroll
      for (int k = 0; k < C::PX; ++k) {
        const int i = tid + 256 * k;
        *reinterpret_cast<float4*>(Xs + h * C::XS + (i >> 2) * C::LD + (i & 3) * 4) = px[h][k];
      }
#pragma unroll
      for (int k = 0; k < C::PW; ++k) {
        int q = tid + 256 * k;
        if (q < C::W4) {
          asm volatile("" : "+v"(q));  // as in convbig_kernel: recompute the destinations, do not hoist them
          int dst[4];
          (void)cb_wsrc<BN, C::LD>(a, n0, 0, q, dst);
          float* w = Ws + h * C::WS;
          w[dst[0]] = pw[h][k].x;
          w[dst[1]] = pw[h][k].y;
          w[dst[2]] = pw[h][k].z;
          w[dst[3]] = pw[h][k].w;
        }
      }
    }
  };

  f32x4 acc[4][WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  for (int s = 0; s < nstage; ++s) {
    __syncthreads();  // every wave is done reading the previous stage
    store();
    __syncthreads();
    if (s + 1 < nstage) load((s + 1) * CB_KC * SPS);  // in flight across this stage's MFMAs
#pragma unroll
    for (int h = 0; h < SPS; ++h) {
      float4 av[4], bv[WN];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        av[i] = *reinterpret_cast<const float4*>(Xs + h * C::XS + (wm * 64 + i * 16 + l16) * C::LD + 4 * lg);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        bv[j] = *reinterpret_cast<const float4*>(Ws + h * C::WS + (wn * (BN / 2) + j * 16 + l16) * C::LD + 4 * lg);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            const float ae = e == 0 ? av[i].x : e == 1 ? av[i].y : e == 2 ? av[i].z : av[i].w;
            const float be = e == 0 ? bv[j].x : e == 1 ? bv[j].y : e == 2 ? bv[j].z : bv[j].w;
            acc[i][j] = mfma16x16x4(ae, be, acc[i][j]);
          }
    }
  }
  cb_epilogue<BN, SOFTMAX>(a, acc, Xs, m0, n0);
}

// shapes the wide kernel takes: PCL in and out, Kc a multiple of 16 (whole slices), N a multiple of 4 (no pad
// channels, whole weight float4s), no CF outputs / fused tails / softmax wider than half a tile
bool convbig_supported(const ConvArgs& a) {
  return !a.src_cf && a.Kc % CB_KC == 0 && a.Kc > 0 && a.N % 4 == 0 && a.N > 0 && (a.ks == 1 || a.ks == 3) &&
         !a.out_cf && !a.tW && !a.t_cf0 && !a.q_cf && !a.reg_out && a.act <= 2 && (a.act != 2 || a.aux) &&
         (!a.q_out || a.N <= 64) && (a.out || a.q_out) && a.R < (1ll << 40);
}

template <int BN, bool SM>
static int launch_cb(const ConvArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)(cdiv(cdiv(a.R, CB_BM), 8) * 8 * cdiv(a.N, BN)));
  if (a.ks == 1 && a.Kc % (CB_KC * ConvBig1Cfg<BN>::SPS) == 0) {
    const size_t lds1 = (size_t)ConvBig1Cfg<BN>::LDS_FLOATS * sizeof(float);
    convbig1_kernel<BN, SM><<<grid, 256, lds1, s>>>(a);
    VQHMM_LAUNCH_CHECK();
    return VQHMM_OK;
  }
  const size_t lds = (size_t)ConvBigCfg<BN>::LDS_FLOATS * sizeof(float);
  convbig_kernel<BN, SM><<<grid, 256, lds, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_convbig(const ConvArgs& a, hipStream_t s) {
  if (!convbig_supported(a)) return VQHMM_EUNSUPPORTED;
  if (a.R == 0) return VQHMM_OK;
  if (a.q_out) return a.N <= 32 ? launch_cb<64, true>(a, s) : launch_cb<128, true>(a, s);  // N <= BN / 2
  if (a.N <= 32) return launch_cb<32, false>(a, s);  // e.g. the dgrad of dec_conv1 into K = 32 states
  // 64-column tiles for every wider layer: ~100 VGPRs against 145 for 128 columns, so more waves per SIMD; that
  // outweighs X being read once per 64 output columns instead of once per 128 (cfg3, one box: k = 3 layers
  // 16.19 -> 15.70 ms; k = 1 layers neutral, 15.70 -> 15.69)
  return launch_cb<64, false>(a, s);
}


// ------------------------------------------------------------------ wide weight gradients
// dW[n][c][tap] = sum_r dY[r][n] X[r + tap - 1][c] over a chunk of PCL rows (split-K; the per-chunk partials go
// to a slab the backward tail sums in a fixed order), and the bias gradient sum_r dY[r][n] (c-tile 0).  A
// workgroup owns TN = 128 outputs n x TC = 64 inputs c x every tap; its 4 waves split that 2 x 2 (64 n x 32 c x
// ks taps: 4 x 2 x ks accumulators).  64-row stages of dY and X (one halo row each side) in LDS, the next stage
// in flight in registers; operands are b32 reads with row strides = 16 (mod 64) floats (the four 16-lane groups
// read rows 4 apart in disjoint banks).
namespace {
constexpr int WB_TN = 128, WB_TC = 64, WB_RT = 64;  // the default tile (the kernel's MI = 4, NJ = 2)
}  // namespace

template <int KS, int MI, int NJ>
__global__ __launch_bounds__(256) void wgradbig_kernel(WgradArgs a) {
  // TN = 32 MI outputs x TC = 32 NJ inputs per workgroup (128 x 64 by default; narrower for N or C <= 32, where
  // the default tile was 1/2 to 3/4 empty): each wave 16 MI x 16 NJ of them
  constexpr int TN = 32 * MI, TC = 32 * NJ, LDA = TN + 16, LDB = TC + 16;  // strides = 16 (mod 64)
  constexpr int DY4 = WB_RT * TN / 4, X4 = (WB_RT + 2) * TC / 4, PD = DY4 / 256, PX = (X4 + 255) / 256;
  __shared__ float dys[WB_RT * LDA];
  __shared__ float xs[(WB_RT + 2) * LDB];
  __shared__ float bred[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg = lane >> 4, l16 = lane & 15;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntc = (int)cdiv(a.C, TC);
  const int n0 = (blockIdx.x / ntc) * TN, c0 = (blockIdx.x % ntc) * TC;
  const int64_t chunk = blockIdx.y;
  const int64_t rbeg = chunk * a.rows_per_chunk, rend = min(a.R, rbeg + a.rows_per_chunk);
  const int ldn = ld4(a.N), ldc = ld4(a.C);
  const bool do_bias = a.bias_slab && c0 == 0;

  float4 pd[PD], px[PX];
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int i = tid + 256 * k, row = i / (TN / 4), n = n0 + (i - row * (TN / 4)) * 4;
      const int64_t r = r0 + row;
      pd[k] = (r < rend && n < ldn) ? *reinterpret_cast<const float4*>(a.dy + r * ldn + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int i = tid + 256 * k, row = i / (TC / 4), c = c0 + (i - row * (TC / 4)) * 4;
      const int64_t r = r0 - 1 + row;
      px[k] = (i < X4 && r >= 0 && r < a.R && c < ldc) ? *reinterpret_cast<const float4*>(a.x + r * ldc + c)
                                                           : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  f32x4 acc[KS][MI][NJ];
#pragma unroll
  for (int tp = 0; tp < KS; ++tp)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[tp][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;

  load(rbeg);
  for (int64_t r0 = rbeg; r0 < rend; r0 += WB_RT) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int i = tid + 256 * k, row = i / (TN / 4), n = (i - row * (TN / 4)) * 4;
      *reinterpret_cast<float4*>(dys + row * LDA + n) = pd[k];
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int i = tid + 256 * k, row = i / (TC / 4), c = (i - row * (TC / 4)) * 4;
      if (i < X4) *reinterpret_cast<float4*>(xs + row * LDB + c) = px[k];
    }
    __syncthreads();
    if (r0 + WB_RT < rend) load(r0 + WB_RT);
    if (do_bias && tid < TN) {
      float bp[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) bp[k] = 0.f;
#pragma unroll
      for (int row = 0; row < WB_RT; ++row) bp[row & 7] += dys[row * LDA + tid];
      bacc += ((bp[0] + bp[1]) + (bp[2] + bp[3])) + ((bp[4] + bp[5]) + (bp[6] + bp[7]));
    }
#pragma unroll 4
    for (int st = 0; st < WB_RT / 4; ++st) {
      const int rr = 4 * st + lg;  // this lane group's row of the k-step
      float av[MI], bv[KS][NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) av[i] = dys[rr * LDA + wm * (TN / 2) + i * 16 + l16];
#pragma unroll
      for (int tp = 0; tp < KS; ++tp)
#pragma unroll
        for (int j = 0; j < NJ; ++j) bv[tp][j] = xs[(rr + (KS == 3 ? tp : 1)) * LDB + wn * (TC / 2) + j * 16 + l16];
#pragma unroll
      for (int tp = 0; tp < KS; ++tp)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[tp][i][j] = mfma16x16x4(av[i], bv[tp][j], acc[tp][i][j]);
    }
  }
  // ---- this chunk's partial: slab[chunk][n][c][tap]; lane (lg, l16), reg v -> n row 4 lg + v, c column l16
  float* out = a.slab + chunk * (int64_t)a.N * a.C * KS;
#pragma unroll
  for (int tp = 0; tp < KS; ++tp)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int n = n0 + wm * (TN / 2) + i * 16 + 4 * lg + v, c = c0 + wn * (TC / 2) + j * 16 + l16;
          if (n < a.N && c < a.C) out[((int64_t)n * a.C + c) * KS + tp] = acc[tp][i][j][v];
        }
  if (do_bias && tid < TN && n0 + tid < a.N) a.bias_slab[chunk * a.N + n0 + tid] = bacc;
  (void)bred;
}

// the wide weight gradients: PCL operands, N and C multiples of 4
bool wgradbig_supported(const WgradArgs& a) {
  return !a.x_cf && a.N % 4 == 0 && a.C % 4 == 0 && a.N > 0 && a.C > 0 && (a.ks == 1 || a.ks == 3) &&
         !a.cmpW && a.rows_per_chunk % WB_RT == 0;
}

// rows per chunk: about 768 workgroups over the output tiles, whole 64-row stages
int64_t wgradbig_rows(int64_t R, int N, int C) {
  const int64_t tiles = cdiv(N, WB_TN) * cdiv(C, WB_TC);
  const int64_t want = std::max<int64_t>(1, 768 / tiles);
  return std::max<int64_t>(WB_RT, cdiv(cdiv(R, want), WB_RT) * WB_RT);
}

int launch_wgradbig(const WgradArgs& a, hipStream_t s) {
  if (!wgradbig_supported(a)) return VQHMM_EUNSUPPORTED;
  if (a.R == 0) return VQHMM_OK;
  const dim3 grid((unsigned)(cdiv(a.N, WB_TN) * cdiv(a.C, WB_TC)), (unsigned)cdiv(a.R, a.rows_per_chunk));
  // narrower tiles only where they keep the default tile count (wgradbig_rows' chunking and the slabs)
  const int mi = a.N <= 32 ? 1 : 4, nj = a.C <= 32 ? 1 : 2;
  if (a.ks == 3) {
    if (mi == 4 && nj == 1) wgradbig_kernel<3, 4, 1><<<grid, 256, 0, s>>>(a);
    else if (mi == 1 && nj == 2) wgradbig_kernel<3, 1, 2><<<grid, 256, 0, s>>>(a);
    else wgradbig_kernel<3, 4, 2><<<grid, 256, 0, s>>>(a);
  } else {
    if (mi == 4 && nj == 1) wgradbig_kernel<1, 4, 1><<<grid, 256, 0, s>>>(a);
    else if (mi == 1 && nj == 2) wgradbig_kernel<1, 1, 2><<<grid, 256, 0, s>>>(a);
    else wgradbig_kernel<1, 4, 2><<<grid, 256, 0, s>>>(a);
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
