// Conv1d (k = 1 or 3, padding = k/2) as an implicit GEMM on fp32 MFMA.
//
// Replaces the ATen work of every Conv1d on the path (SURVEY.md §8a A1-A3,
// A5-A7, A11): Encoder.conv1/conv2/to_logits (VQ_VAE_HMM_fixed.py:34-36,39-41),
// Decoder.conv1/conv2/to_params (:77-79,85-87), and their autograd backward.
//
// GEMM view over PCL rows (see common.h): Y[r, n] = sum_{tap, c} X[r + tap - 1, c] * Weff[n, c, tap].
// The zero pad rows of the PCL layout make the im2col implicit and mask-free.
//
//  conv_mm_kernel   forward (Weff = W) and data-gradient (Weff[n,c,tap] =
//                   W[c,n,k-1-tap]: the transposed, flipped weight) in one
//                   kernel, with a fused epilogue: grad scale, bias, ReLU or
//                   ReLU-backward mask, pad-row zeroing, PCL and/or CF stores,
//                   and an optional fused 1x1 "tail" conv (+softmax) on the
//                   activated tile (to_logits / to_params).
//  wgrad_kernel     weight/bias gradient as a split-K GEMM over rows; every
//                   workgroup writes its partial into a slab, summed later in
//                   a fixed order (deterministic, no atomics).
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32).  Per K=16 slice each lane reads
// one float4 of A and one of B from LDS and issues 4 MFMAs per 16x16 block;
// the k index inside a slice is permuted (lane group g, element e <-> channel
// 4g+e) identically for A and B, so the sum is unchanged.
#include "kernels.h"

namespace vqhmm {


__device__ __forceinline__ float weff(const ConvArgs& a, int n, int c, int tap) {
  if (!a.w_dgrad) return a.W[((int64_t)n * a.Kc + c) * a.ks + tap];
  return a.W[((int64_t)c * a.N + n) * a.ks + (a.ks - 1 - tap)];
}

template <int WAVES_M, int WAVES_N, int WM, int WN, int KCH>
__global__ __launch_bounds__(256) void conv_mm_kernel(ConvArgs a) {
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  constexpr int LDX = KCH + 4;
  constexpr int LDY = BN + 4;
  extern __shared__ float4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  float* Xs = smem;                       // [(BM + 2)][LDX]
  float* Ws = smem + (BM + 2) * LDX;      // [ks][BN][LDX]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int64_t Tp = (int64_t)a.T + 2;

  f32x4 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool vec_src = !a.src_cf;  // PCL rows have stride ld4(Kc): always float4-aligned
  const int lds = ld4(a.Kc);
  for (int c0 = 0; c0 < a.Kc; c0 += KCH) {
    __syncthreads();
    // ---- stage input rows [m0-1, m0+BM] x channels [c0, c0+KCH)
    if (a.src_cf) {
      for (int i = tid; i < (BM + 2) * KCH; i += 256) {
        const int row = i % (BM + 2), c = i / (BM + 2);
        const int64_t r = m0 - 1 + row;
        float v = 0.f;
        if (r >= 0 && r < a.R && c0 + c < a.Kc) {
          const int64_t b = r / Tp;
          const int t = (int)(r - b * Tp) - 1;
          if (t >= 0 && t < a.T) v = a.src[(b * a.Kc + c0 + c) * a.T + t];
        }
        Xs[row * LDX + c] = v;
      }
    } else if (vec_src) {
      for (int i = tid; i < (BM + 2) * (KCH / 4); i += 256) {
        const int row = i / (KCH / 4), c = (i - row * (KCH / 4)) * 4;
        const int64_t r = m0 - 1 + row;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r >= 0 && r < a.R && c0 + c < lds) v = *reinterpret_cast<const float4*>(a.src + r * lds + c0 + c);
        *reinterpret_cast<float4*>(Xs + row * LDX + c) = v;
      }
    } else {
      for (int i = tid; i < (BM + 2) * KCH; i += 256) {
        const int row = i / KCH, c = i - row * KCH;
        const int64_t r = m0 - 1 + row;
        float v = 0.f;
        if (r >= 0 && r < a.R && c0 + c < a.Kc) v = a.src[r * lds + c0 + c];
        Xs[row * LDX + c] = v;
      }
    }
    // ---- stage weights Ws[tap][n][c]
    for (int i = tid; i < a.ks * BN * KCH; i += 256) {
      const int c = i % KCH, n = (i / KCH) % BN, tap = i / (KCH * BN);
      float v = 0.f;
      if (n0 + n < a.N && c0 + c < a.Kc) v = weff(a, n0 + n, c0 + c, tap);
      Ws[(tap * BN + n) * LDX + c] = v;
    }
    __syncthreads();
    // ---- MFMA main loop
    for (int tap = 0; tap < a.ks; ++tap) {
      const int rowoff = (a.ks == 3) ? tap : 1;
#pragma unroll
      for (int kk = 0; kk < KCH / 16; ++kk) {
        const int col = kk * 16 + 4 * (lane >> 4);
        float4 av[WM], bv[WN];
#pragma unroll
        for (int i = 0; i < WM; ++i)
          av[i] = *reinterpret_cast<const float4*>(Xs + (wm * WM * 16 + i * 16 + (lane & 15) + rowoff) * LDX + col);
#pragma unroll
        for (int j = 0; j < WN; ++j)
          bv[j] = *reinterpret_cast<const float4*>(Ws + (tap * BN + wn * WN * 16 + j * 16 + (lane & 15)) * LDX + col);
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            acc[i][j] = mfma16x16x4(av[i].x, bv[j].x, acc[i][j]);
            acc[i][j] = mfma16x16x4(av[i].y, bv[j].y, acc[i][j]);
            acc[i][j] = mfma16x16x4(av[i].z, bv[j].z, acc[i][j]);
            acc[i][j] = mfma16x16x4(av[i].w, bv[j].w, acc[i][j]);
          }
      }
    }
  }

  // ---------------------------------------------------------------- epilogue
  __syncthreads();
  float* Ys = smem;  // [BM][LDY]
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = wm * WM * 16 + i * 16 + (lane >> 4) * 4 + v;
        const int col = wn * WN * 16 + j * 16 + (lane & 15);
        Ys[row * LDY + col] = acc[i][j][v];
      }
  __syncthreads();
  const float sc = a.scale ? *a.scale : 1.0f;
  // four elements per thread and pass, their bias / mask loads issued before any of their stores (a load after
  // a store to `out`, which may alias it as far as the compiler knows, was issued and waited for alone)
  constexpr int EP = 4;
  for (int i0 = tid; i0 < BM * BN; i0 += 256 * EP) {
    float bv[EP], mv[EP];
#pragma unroll
    for (int u = 0; u < EP; ++u) {
      const int i = i0 + 256 * u, row = i / BN, n = n0 + (i - row * BN);
      const int64_t r = m0 + row;
      const bool in = i < BM * BN && n < a.N && r < a.R;
      bv[u] = in && a.bias ? a.bias[n] : 0.f;
      mv[u] = in && a.act == 2 ? a.aux[r * ld4(a.N) + n] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < EP; ++u) {
      const int i = i0 + 256 * u;
      if (i >= BM * BN) break;
      const int row = i / BN, col = i - row * BN;
      const int64_t r = m0 + row;
      const int n = n0 + col;
      float y = 0.f;
      int64_t b;
      int t;
      if (n < a.N && row_bt_fast(r, a.R, a.T, b, t)) {
        y = Ys[row * LDY + col] * sc;
        if (a.bias) y += bv[u];
        if (a.act == 1) y = relu_f(y);
        else if (a.act == 2) y = mv[u] > 0.f ? y : 0.f;
      }
      Ys[row * LDY + col] = y;
      if (a.out && n < ld4(a.N) && r < a.R) a.out[r * ld4(a.N) + n] = y;
    }
  }
  if (a.out_cf || a.tW) __syncthreads();
  if (a.out_cf) {
    for (int i = tid; i < BM * BN; i += 256) {
      const int row = i % BM, col = i / BM;
      const int64_t r = m0 + row;
      const int n = n0 + col;
      int64_t b;
      int t;
      if (n < a.N && row_bt(r, a.R, a.T, b, t)) a.out_cf[(b * a.N + n) * a.T + t] = Ys[row * LDY + col];
    }
  }
  if (!a.tW) return;
  // ---- fused 1x1 tail: z = tW @ y + tb (and softmax over C2), thread per row
  float* Zs = smem + BM * LDY;  // [BM][C2 + 1]
  const int LDZ = a.C2 + 1;
  for (int row = tid; row < BM; row += 256) {
    const int64_t r = m0 + row;
    int64_t b;
    int t;
    const bool valid = row_bt(r, a.R, a.T, b, t);
    float mx = -__builtin_inff();
    for (int c2 = 0; c2 < a.C2; ++c2) {
      float z = 0.f;
      if (valid) {
        z = a.tb ? a.tb[c2] : 0.f;
        const float* w = a.tW + (int64_t)c2 * a.N;
        for (int n = 0; n < a.N; ++n) z = fmaf(w[n], Ys[row * LDY + n], z);
      }
      Zs[row * LDZ + c2] = z;
      mx = fmaxf(mx, z);
      if (a.t_out && r < a.R) a.t_out[r * ld4(a.C2) + c2] = z;
    }
    for (int c2 = a.C2; c2 < ld4(a.C2); ++c2) {
      if (a.t_out && r < a.R) a.t_out[r * ld4(a.C2) + c2] = 0.f;
      if (a.q_out && r < a.R) a.q_out[r * ld4(a.C2) + c2] = 0.f;
    }
    if (a.q_out || a.q_cf || a.reg_out) {
      float s = 0.f;
      for (int c2 = 0; c2 < a.C2; ++c2) s += __expf(Zs[row * LDZ + c2] - mx);
      float bq = -__builtin_inff();
      int bi = 0x7fffffff;
      for (int c2 = 0; c2 < a.C2; ++c2) {
        const float q = valid ? __expf(Zs[row * LDZ + c2] - mx) / s : 0.f;
        if (a.q_out && r < a.R) a.q_out[r * ld4(a.C2) + c2] = q;
        if (a.q_cf) Zs[row * LDZ + c2] = q;
        if (argmax_beats(q, c2, bq, bi)) { bq = q; bi = c2; }
      }
      if (a.reg_out && valid) a.reg_out[b * a.T + t] = bi;  // hard regime (backtesting.py:154-155)
    }
  }
  if (a.t_cf0 || a.q_cf) {
    __syncthreads();
    for (int i = tid; i < BM * a.C2; i += 256) {
      const int row = i % BM, c2 = i / BM;
      const int64_t r = m0 + row;
      int64_t b;
      int t;
      if (!row_bt(r, a.R, a.T, b, t)) continue;
      const float v = Zs[row * LDZ + c2];
      if (a.q_cf) {
        a.q_cf[(b * a.C2 + c2) * a.T + t] = v;
      } else if (c2 < a.t_split) {
        a.t_cf0[(b * a.t_split + c2) * a.T + t] = v;
      } else {
        const int ns = a.C2 - a.t_split;
        a.t_cf1[(b * ns + c2 - a.t_split) * a.T + t] = v;
      }
    }
  }
}

template <int WAVES_M, int WAVES_N, int WM, int WN, int KCH>
static int launch_conv_cfg(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  const size_t main_lds = ((size_t)(BM + 2) * (KCH + 4) + (size_t)a.ks * BN * (KCH + 4)) * 4;
  size_t epi_lds = (size_t)BM * (BN + 4) * 4;
  if (a.tW) epi_lds += (size_t)BM * (a.C2 + 1) * 4;
  const size_t lds = main_lds > epi_lds ? main_lds : epi_lds;
  if (lds > 160 * 1024) return VQHMM_EUNSUPPORTED;
  if (a.tW && a.N > BN) return VQHMM_EUNSUPPORTED;
  const dim3 grid((unsigned)cdiv(a.R, BM), (unsigned)cdiv(a.N, BN));
  conv_mm_kernel<WAVES_M, WAVES_N, WM, WN, KCH><<<grid, 256, lds, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// The wide-channel path (convbig.hip): the conv on convbig_kernel and a fused 1x1 tail (to_logits + softmax,
// to_params) as a second convbig launch over the activation the first one stored.  Null when it does not apply.
static bool convbig_split(const ConvArgs& a, ConvArgs& main, ConvArgs& tail) {
  main = a;
  main.tW = nullptr; main.tb = nullptr; main.C2 = 0; main.t_out = nullptr; main.q_out = nullptr;
  if (!convbig_supported(main)) return false;
  if (!a.tW) return !a.q_out;
  if (!a.out || !a.t_out || a.t_cf0 || a.q_cf || a.reg_out) return false;
  tail = ConvArgs{};
  tail.R = a.R; tail.T = a.T;
  tail.src = a.out; tail.Kc = a.N; tail.ks = 1; tail.W = a.tW; tail.bias = a.tb; tail.N = a.C2; tail.act = 0;
  tail.out = a.t_out; tail.q_out = a.q_out;
  return convbig_supported(tail);
}

int launch_conv(const ConvArgs& a, hipStream_t s) {
  if (a.R == 0) return VQHMM_OK;
  if (!a.src || !a.W || a.Kc <= 0 || a.N <= 0 || (a.ks != 1 && a.ks != 3)) return VQHMM_EINVAL;
  if (conv2_supported(a)) return launch_conv2(a, s);
  ConvArgs cm, ct;
  if (convbig_split(a, cm, ct)) {
    if (int rc = launch_convbig(cm, s)) return rc;
    return a.tW ? launch_convbig(ct, s) : VQHMM_OK;
  }
  const bool wide = a.Kc > 16;
  if (a.N <= 16) return wide ? launch_conv_cfg<4, 1, 4, 1, 32>(a, s) : launch_conv_cfg<4, 1, 4, 1, 16>(a, s);
  if (a.N <= 32) return wide ? launch_conv_cfg<4, 1, 4, 2, 32>(a, s) : launch_conv_cfg<4, 1, 4, 2, 16>(a, s);
  if (a.N <= 64) return wide ? launch_conv_cfg<2, 2, 4, 2, 32>(a, s) : launch_conv_cfg<2, 2, 4, 2, 16>(a, s);
  if (a.N <= 128) return wide ? launch_conv_cfg<1, 4, 4, 2, 32>(a, s) : launch_conv_cfg<1, 4, 4, 2, 16>(a, s);
  return launch_conv_cfg<1, 4, 4, 4, 16>(a, s);
}

// ------------------------------------------------------------------ wgrad

// 4 waves as 2x2; each wave owns a (16*WM) x (16*WN) block of (n, c) for every tap.
template <int WM, int WN>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs a) {
  constexpr int TN = 2 * WM * 16, TC = 2 * WN * 16;  // workgroup output tile
  constexpr int RT = 64;                              // rows per LDS stage
  constexpr int LDA = TN + 4, LDB = TC + 4;           // stride = 4 (mod 8) floats -> conflict-free b32 reads
  __shared__ float dys[RT * LDA];
  __shared__ float xs[(RT + 2) * LDB];
  __shared__ float bsum[4][TN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles_c = (int)cdiv(a.C, TC);
  const int n0 = (blockIdx.x / ntiles_c) * TN;
  const int c0 = (blockIdx.x % ntiles_c) * TC;
  const int64_t chunk = blockIdx.y;
  const int64_t rbeg = chunk * a.rows_per_chunk;
  const int64_t rend = min(a.R, rbeg + a.rows_per_chunk);
  const int64_t Tp = (int64_t)a.T + 2;
  const bool do_bias = a.bias_slab && c0 == 0;

  f32x4 acc[3][WM][WN];
#pragma unroll
  for (int tp = 0; tp < 3; ++tp)
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[tp][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;

  for (int64_t r0 = rbeg; r0 < rend; r0 += RT) {
    __syncthreads();
    for (int i = tid; i < RT * TN; i += 256) {
      const int row = i / TN, n = i - row * TN;
      const int64_t r = r0 + row;
      dys[row * LDA + n] = (r < rend && n0 + n < a.N) ? a.dy[r * ld4(a.N) + n0 + n] : 0.f;
    }
    if (a.x_cf) {
      for (int i = tid; i < (RT + 2) * TC; i += 256) {
        const int row = i % (RT + 2), c = i / (RT + 2);
        const int64_t r = r0 - 1 + row;
        float v = 0.f;
        if (r >= 0 && r < a.R && c0 + c < a.C) {
          const int64_t b = r / Tp;
          const int t = (int)(r - b * Tp) - 1;
          if (t >= 0 && t < a.T) v = a.x[(b * a.C + c0 + c) * a.T + t];
        }
        xs[row * LDB + c] = v;
      }
    } else {
      for (int i = tid; i < (RT + 2) * TC; i += 256) {
        const int row = i / TC, c = i - row * TC;
        const int64_t r = r0 - 1 + row;
        xs[row * LDB + c] = (r >= 0 && r < a.R && c0 + c < a.C) ? a.x[r * ld4(a.C) + c0 + c] : 0.f;
      }
    }
    __syncthreads();
    if (do_bias && tid < TN) {
      for (int row = 0; row < RT; ++row) bacc += dys[row * LDA + tid];
    }
#pragma unroll
    for (int kk = 0; kk < RT / 16; ++kk) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = kk * 16 + 4 * (lane >> 4) + e;
        float av[WM];
#pragma unroll
        for (int i = 0; i < WM; ++i) av[i] = dys[rr * LDA + wm * WM * 16 + i * 16 + (lane & 15)];
#pragma unroll
        for (int tp = 0; tp < 3; ++tp) {
          if (tp < a.ks) {
            const int xrow = rr + (a.ks == 3 ? tp : 1);
#pragma unroll
            for (int j = 0; j < WN; ++j) {
              const float bvv = xs[xrow * LDB + wn * WN * 16 + j * 16 + (lane & 15)];
#pragma unroll
              for (int i = 0; i < WM; ++i) acc[tp][i][j] = mfma16x16x4(av[i], bvv, acc[tp][i][j]);
            }
          }
        }
      }
    }
  }
  // ---- write this chunk's partial: slab[chunk][n][c][tap]
  float* out = a.slab + chunk * (int64_t)a.N * a.C * a.ks;
#pragma unroll
  for (int tp = 0; tp < 3; ++tp) {
    if (tp >= a.ks) continue;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int n = n0 + wm * WM * 16 + i * 16 + (lane >> 4) * 4 + v;
          const int c = c0 + wn * WN * 16 + j * 16 + (lane & 15);
          if (n < a.N && c < a.C) out[((int64_t)n * a.C + c) * a.ks + tp] = acc[tp][i][j][v];
        }
  }
  if (do_bias) {
    if (tid < TN) bsum[0][tid] = bacc;
    __syncthreads();
    if (tid < TN && n0 + tid < a.N) a.bias_slab[chunk * a.N + n0 + tid] = bsum[0][tid];
  }
}

int64_t wgrad_chunks(int64_t R, int64_t tiles) {
  // aim for ~512 workgroups in total, at least 64 rows per chunk
  int64_t want = (512 + tiles - 1) / tiles;
  int64_t rows = cdiv(R, want);
  rows = cdiv(rows, 64) * 64;
  if (rows < 64) rows = 64;
  return rows;
}

int launch_wgrad(const WgradArgs& a0, hipStream_t s) {
  WgradArgs a = a0;
  if (a.R == 0) return VQHMM_OK;
  if (!a.dy || !a.x || !a.slab || (a.ks != 1 && a.ks != 3) || a.rows_per_chunk % 64) return VQHMM_EINVAL;
  if (wgrad2_supported(a)) return launch_wgrad2(a, s);
  if (wgradbig_supported(a)) return launch_wgradbig(a, s);
  const int64_t nchunks = cdiv(a.R, a.rows_per_chunk);
  constexpr int TN = 64, TC = 64;
  const dim3 grid((unsigned)(cdiv(a.N, TN) * cdiv(a.C, TC)), (unsigned)nchunks);
  wgrad_kernel<2, 2><<<grid, 256, 0, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
