// Device building blocks of the conv2 kernels (conv2.hip) shared with the strip kernels (strip.hip):
// the MFMA tile loops, the epilogue and the per-launch tile configurations.  Header-only so both
// translation units compile the very same instruction sequences (bit-identical results).
#pragma once
#include "kernels.h"

namespace vqhmm {

namespace {

template <int NB, int KCP, int KS, int PB>
struct C2Cfg {
  static constexpr int BM = 4 * PB * 16;       // rows per tile
  static constexpr int KCW = KCP * 16;         // padded input channels
  static constexpr int LDX = KCW + 8;          // LDS row stride = c2_ldx: conflict-free b128 reads
  static constexpr int NW = NB * 16;           // padded output channels
  static constexpr int XROWS = BM + 2;
  static constexpr int XF4 = XROWS * KCW / 4;  // float4 slots of one X tile
  static constexpr int PF = (XF4 + 255) / 256; // float4 slots per thread
  static constexpr size_t W_FLOATS = (size_t)KS * NW * LDX;
  static constexpr size_t X_FLOATS = (size_t)XROWS * LDX;
  static constexpr size_t LDS = (W_FLOATS + X_FLOATS) * 4;
};

// Raw float4 slot `s` of an X tile starting at PCL row m0-1 (row stride
// ld4(Kc)): the address is clamped in range and x_mask() zeroes what lies
// outside the tile's rows / the row's channels afterwards — keeping the select
// away from the load lets the prefetch stay in flight across the MFMA loop.
__device__ __forceinline__ float4 x_raw(const ConvArgs& a, int64_t m0, int s, int kcw) {
  const int q4 = kcw / 4, ld = ld4(a.Kc);
  const int row = s / q4, c = (s - row * q4) * 4;
  int64_t r = m0 - 1 + row;
  r = r < 0 ? 0 : (r >= a.R ? a.R - 1 : r);
  return *reinterpret_cast<const float4*>(a.src + r * ld + min(c, ld - 4));
}

__device__ __forceinline__ float4 x_mask(const ConvArgs& a, int64_t m0, int s, int kcw, float4 v) {
  const int q4 = kcw / 4;
  const int row = s / q4, c = (s - row * q4) * 4;
  const int64_t r = m0 - 1 + row;
  const bool ok = r >= 0 && r < a.R && c < ld4(a.Kc);  // pad channels inside the row are already 0
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

}  // namespace

// The tile's MFMAs: acc[nb][pb] (16 n x 16 rows) += W_tap (n x c) @ X(rows + tap - 1, c)^T over the
// KS * KCP 16-wide k-steps.  Operands of step s + 1 are read from LDS while the 16*PB MFMAs of step
// s run (two register sets; sched_barrier keeps the reads ahead of the MFMAs), and the MFMAs are
// issued component-major so consecutive ones use different accumulators (the accumulator chain
// of every block is still x, y, z, w per step: the same k-ordered fma chain as before).
// Xw = row 0 of the wave's first 16-row block in the X tile (tile row 0 = PCL row m0 - 1).
template <int NB, int PB, int KCP, int KS, int LDX, int NW>
__device__ __forceinline__ void c2_mfma_tile(const float* Ws, const float* Xw, int lg4, int l16,
                                             f32x4 (&acc)[NB][PB], bool pipe) {
  constexpr int NSTEP = KS * KCP;
  if (!pipe) {  // A/B reference: operands read per step, accumulator-major issue
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      const int tap = st / KCP, kk = st - tap * KCP;
      const int rowoff = (KS == 3) ? tap : 1;
      const int col = kk * 16 + 4 * lg4;
      float4 a[NB], b[PB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        a[nb] = *reinterpret_cast<const float4*>(Ws + (tap * NW + nb * 16 + l16) * LDX + col);
#pragma unroll
      for (int pb = 0; pb < PB; ++pb)
        b[pb] = *reinterpret_cast<const float4*>(Xw + (pb * 16 + l16 + rowoff) * LDX + col);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int pb = 0; pb < PB; ++pb) {
          acc[nb][pb] = mfma16x16x4(a[nb].x, b[pb].x, acc[nb][pb]);
          acc[nb][pb] = mfma16x16x4(a[nb].y, b[pb].y, acc[nb][pb]);
          acc[nb][pb] = mfma16x16x4(a[nb].z, b[pb].z, acc[nb][pb]);
          acc[nb][pb] = mfma16x16x4(a[nb].w, b[pb].w, acc[nb][pb]);
        }
    }
    return;
  }
  float4 av[2][NB], bv[2][PB];
  auto load = [&](int st, float4 (&a)[NB], float4 (&b)[PB]) {
    const int tap = st / KCP, kk = st - tap * KCP;
    const int rowoff = (KS == 3) ? tap : 1;
    const int col = kk * 16 + 4 * lg4;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      a[nb] = *reinterpret_cast<const float4*>(Ws + (tap * NW + nb * 16 + l16) * LDX + col);
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
      b[pb] = *reinterpret_cast<const float4*>(Xw + (pb * 16 + l16 + rowoff) * LDX + col);
  };
  load(0, av[0], bv[0]);
#pragma unroll
  for (int st = 0; st < NSTEP; ++st) {
    const int cb = st & 1;
    if (st + 1 < NSTEP) load(st + 1, av[cb ^ 1], bv[cb ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int pb = 0; pb < PB; ++pb) {
          const float x = e == 0 ? av[cb][nb].x : e == 1 ? av[cb][nb].y : e == 2 ? av[cb][nb].z : av[cb][nb].w;
          const float y = e == 0 ? bv[cb][pb].x : e == 1 ? bv[cb][pb].y : e == 2 ? bv[cb][pb].z : bv[cb][pb].w;
          acc[nb][pb] = mfma16x16x4(x, y, acc[nb][pb]);
        }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Packed taps for a narrow k = 3 layer (3 * Kc <= 16): k-column j = tap * Kc + c, so the three taps
// share ONE 16-wide k-block — NB x 4 MFMAs per 16 rows instead of 3 x NB x 4.  Operands are per-lane
// gathers from the standard weight image [tap][n][LDX] and X slot [row][LDX]; columns past 3 * Kc
// read tap 0's zero pad column 15 (image and slot are zero past the layer's channels).
template <int NB, int LDX, int NW>
__device__ __forceinline__ void c2_mfma_pk(const float* Ws, const float* Xw, int lg4, int l16, int C,
                                           f32x4 (&acc)[NB][1]) {
  int wo[4], xo[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = 4 * lg4 + e;
    const bool in = k < 3 * C;
    const int tap = in ? k / C : 0, c = in ? k - tap * C : 15;
    wo[e] = (tap * NW + l16) * LDX + c;
    xo[e] = (l16 + tap) * LDX + c;
  }
  float b[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) b[e] = Xw[xo[e]];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    float a4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) a4[e] = Ws[wo[e] + nb * 16 * LDX];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[nb][0] = mfma16x16x4(a4[e], b[e], acc[nb][0]);
  }
}

// Epilogue of one tile (ACT: 0 none, 1 ReLU, 2 ReLU-backward mask by aux, 3 none + the softmax
// backward of the row, see ConvArgs::lb_*).
// Rows of a 16-row block outside [rlo, rhi) get their values (acc) but no stores: the fused
// front conv's halo rows and the rows past a 14-row fused tile belong to the neighbouring tiles.
// xs_q (strip kernels): the softmax q of every row of the block, halo rows included, also goes to LDS
// rows xs_q + l16 * xs_q_ld (channels c0 < xs_q_ld).
// TB = 2: a second 16-channel tail block (channels 16 .. C2-1, C2 <= 32: to_params at D <= 16) with
// weights tw2 / bias tb1; no softmax outputs then.
// xs_dl (ACT 3, strip_bwdw): the row's softmax-backward output dl[0..3] also goes to LDS row xs_dl + 8 l16
// (zeros for rows outside [0, R)).
template <int NB, int PB, int ACT, int TB = 1>
__device__ __forceinline__ void conv2_epilogue(const ConvArgs& a, int64_t m0, int wave, int lg4, int l16,
                                               f32x4 (&acc)[NB][PB], const float4 (&auxv)[NB][PB],
                                               const float (&bias_r)[NB][4], const float (&tw)[NB][4],
                                               f32x4 tb0, float sc, bool tail, int rlo = 0, int rhi = 16,
                                               float* xs_dh = nullptr, int xs_ld = 0,
                                               const float (*tw2)[4] = nullptr, f32x4 tb1 = f32x4{0.f, 0.f, 0.f, 0.f},
                                               float* xs_q = nullptr, int xs_q_ld = 0, float* xs_dl = nullptr) {
  // lane (lg4, l16) holds channels nb*16 + 4*lg4 + v of row m0 + (wave*PB+pb)*16 + l16
  const bool own = l16 >= rlo && l16 < rhi;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      const int64_t r = m0 + (wave * PB + pb) * 16 + l16;
      int64_t b;
      int t;
      const bool valid = row_bt(r, a.R, a.T, b, t);
      const bool st_r = own && r < a.R;  // this row is stored (PCL)
      const bool st_v = own && valid;    // ... and is a valid position (CF)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        f32x4 y;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float yy = acc[nb][pb][v] * sc + bias_r[nb][v];
          if (ACT == 1) yy = relu_f(yy);
          if (ACT == 2) {
            const float av = v == 0 ? auxv[nb][pb].x : v == 1 ? auxv[nb][pb].y : v == 2 ? auxv[nb][pb].z : auxv[nb][pb].w;
            yy = av > 0.f ? yy : 0.f;
          }
          y[v] = valid ? yy : 0.f;
        }
        acc[nb][pb] = y;
        const int n0 = nb * 16 + 4 * lg4;
        if constexpr (ACT == 3 || ACT == 4) {  // softmax backward of the row, then (optionally) to_logits' dgrad
          // ACT 3: K <= 4 channels (one lane group), ACT 4: K <= 8 (lane groups 0 and 1)
          constexpr int KM = ACT == 4 ? 8 : 4;
          if (nb == 0) {
            // channels 0..3 of row l16 sit in lane l16 (lg4 = 0), 4..7 in lane 16 + l16 (lg4 = 1):
            // broadcast them to the row's lanes
            float yk[KM];
#pragma unroll
            for (int k = 0; k < 4; ++k) yk[k] = __shfl(y[k], l16);
            if constexpr (KM == 8) {
#pragma unroll
              for (int k = 0; k < 4; ++k) yk[4 + k] = __shfl(y[k], 16 + l16);
            }
            // rows inside [0, R) are computed (a fused next conv's halo rows need them, xs_dh),
            // only owned rows are stored
            if (r >= 0 && r < a.R) {
              const float lsc = a.lb_scale ? *a.lb_scale : 1.f;
              float qk[KM], xk[KM], lk[KM];
#pragma unroll
              for (int h = 0; h < KM / 4; ++h) {
                const float4 q4 = *reinterpret_cast<const float4*>(a.lb_q + r * KM + 4 * h);
                const float4 x4 = *reinterpret_cast<const float4*>(a.lb_dqx + r * KM + 4 * h);
                const float4 l4 = *reinterpret_cast<const float4*>(a.lb_dlx + r * KM + 4 * h);
                qk[4 * h] = q4.x; qk[4 * h + 1] = q4.y; qk[4 * h + 2] = q4.z; qk[4 * h + 3] = q4.w;
                xk[4 * h] = x4.x; xk[4 * h + 1] = x4.y; xk[4 * h + 2] = x4.z; xk[4 * h + 3] = x4.w;
                lk[4 * h] = l4.x; lk[4 * h + 1] = l4.y; lk[4 * h + 2] = l4.z; lk[4 * h + 3] = l4.w;
              }
              float dq[KM], sdot = 0.f;
#pragma unroll
              for (int k = 0; k < KM; ++k) {
                dq[k] = yk[k] + lsc * xk[k];
                sdot = fmaf(qk[k], dq[k], sdot);
              }
              float dl[KM];
#pragma unroll
              for (int k = 0; k < KM; ++k) dl[k] = qk[k] * (dq[k] - sdot) + lsc * lk[k];
              if (lg4 < KM / 4 && st_r) {
                f32x4 o4;
#pragma unroll
                for (int v = 0; v < 4; ++v) o4[v] = lg4 == 0 ? dl[v] : dl[(4 + v) % KM];
                *reinterpret_cast<f32x4*>(a.lb_dlog + r * KM + 4 * lg4) = o4;
              }
              if (xs_dl && lg4 == 0) *reinterpret_cast<f32x4*>(xs_dl + l16 * 8) = f32x4{dl[0], dl[1], dl[2], dl[3]};
              if (a.lb_dh) {
                // dh[r][c] = (h[r][c] > 0) * sum_k W[k][c] dl[k]: to_logits (1x1, K -> C) dgrad with the
                // ReLU mask of its input h, the same k-ordered fma chain as the MFMA path; lane group
                // lg4 takes channels [lg4 * L / 4, (lg4 + 1) * L / 4) of the ld4(C) = L row
                const int C = a.lb_C, L = ld4(C), per = L / 4;
                for (int c0 = lg4 * per; c0 < (lg4 + 1) * per; c0 += 4) {
                  const float4 h4 = *reinterpret_cast<const float4*>(a.lb_h + r * L + c0);
                  const float hv[4] = {h4.x, h4.y, h4.z, h4.w};
                  f32x4 o;
#pragma unroll
                  for (int v = 0; v < 4; ++v) {
                    const int c = c0 + v;
                    float sacc = 0.f;
#pragma unroll
                    for (int k = 0; k < KM; ++k) sacc = fmaf(c < C && k < a.N ? a.lb_W[k * C + c] : 0.f, dl[k], sacc);
                    o[v] = hv[v] > 0.f ? sacc : 0.f;
                  }
                  if (st_r) *reinterpret_cast<f32x4*>(a.lb_dh + r * L + c0) = o;
                  if (xs_dh) *reinterpret_cast<f32x4*>(xs_dh + l16 * xs_ld + c0) = o;
                }
              }
            } else {
              if (xs_dh && a.lb_dh) {  // rows outside [0, R): the zero padding of the next conv
                const int L = ld4(a.lb_C), per = L / 4;
                for (int c0 = lg4 * per; c0 < (lg4 + 1) * per; c0 += 4)
                  *reinterpret_cast<f32x4*>(xs_dh + l16 * xs_ld + c0) = f32x4{0.f, 0.f, 0.f, 0.f};
              }
              if (xs_dl && lg4 == 0) *reinterpret_cast<f32x4*>(xs_dl + l16 * 8) = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
        if (a.out && st_r && n0 < ld4(a.N)) *reinterpret_cast<f32x4*>(a.out + r * ld4(a.N) + n0) = y;
        if (a.out_cf && st_v) {
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (n0 + v < a.N) a.out_cf[(b * a.N + n0 + v) * a.T + t] = y[v];
        }
      }
      if (tail) {  // compile-time in every caller
#pragma unroll
        for (int tbk = 0; tbk < TB; ++tbk) {
        // z^T (16 c2 x 16 rows) = tW (16 x N) @ Y^T: B operand = the fragments above
        f32x4 z = tbk == 0 ? tb0 : tb1;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int v = 0; v < 4; ++v) z = mfma16x16x4(tbk == 0 ? tw[nb][v] : tw2[nb][v], acc[nb][pb][v], z);
        // lane holds c2 = 16 tbk + 4*lg4 + v of row r
        const int c0 = 16 * tbk + 4 * lg4;
#pragma unroll
        for (int v = 0; v < 4; ++v) z[v] = valid ? z[v] : 0.f;
        if (a.t_out && st_r && c0 < ld4(a.C2)) *reinterpret_cast<f32x4*>(a.t_out + r * ld4(a.C2) + c0) = z;
        if (a.t_cf0 && st_v) {
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int c2 = c0 + v;
            if (c2 < a.t_split) a.t_cf0[(b * a.t_split + c2) * a.T + t] = z[v];
            else if (c2 < a.C2) a.t_cf1[(b * (a.C2 - a.t_split) + c2 - a.t_split) * a.T + t] = z[v];
          }
        }
        if (TB == 1 && (a.q_out || a.q_cf || a.reg_out)) {
          float m = -__builtin_inff();
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (c0 + v < a.C2) m = fmaxf(m, z[v]);
          m = fmaxf(m, __shfl_xor(m, 16));
          m = fmaxf(m, __shfl_xor(m, 32));
          float e[4], s = 0.f;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            e[v] = (c0 + v < a.C2) ? __expf(z[v] - m) : 0.f;
            s += e[v];
          }
          s += __shfl_xor(s, 16);
          s += __shfl_xor(s, 32);
          f32x4 qv;
#pragma unroll
          for (int v = 0; v < 4; ++v) qv[v] = valid ? e[v] / s : 0.f;  // 0 in pad channels (e = 0)
          if (a.q_out && st_r && c0 < ld4(a.C2)) *reinterpret_cast<f32x4*>(a.q_out + r * ld4(a.C2) + c0) = qv;
          // strip kernels: every row's q (halo rows included) into the next conv's LDS input rows
          if (xs_q && c0 < xs_q_ld) *reinterpret_cast<f32x4*>(xs_q + l16 * xs_q_ld + c0) = qv;
          if (a.q_cf && st_v) {
#pragma unroll
            for (int v = 0; v < 4; ++v)
              if (c0 + v < a.C2) a.q_cf[(b * a.C2 + c0 + v) * a.T + t] = qv[v];
          }
          if (a.reg_out) {  // hard regime: first argmax of the row's q (backtesting.py:154-155)
            float bq = -__builtin_inff();
            int bi = 0x7fffffff;
#pragma unroll
            for (int v = 0; v < 4; ++v)
              if (c0 + v < a.C2 && argmax_beats(qv[v], c0 + v, bq, bi)) { bq = qv[v]; bi = c0 + v; }
#pragma unroll
            for (int o = 16; o <= 32; o <<= 1) {
              const float pq = __shfl_xor(bq, o);
              const int pi = __shfl_xor(bi, o);
              if (argmax_beats(pq, pi, bq, bi)) { bq = pq; bi = pi; }
            }
            if (st_v && lg4 == 0) a.reg_out[b * a.T + t] = bi;
          }
        }
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Wave-independent variant: the workgroup (up to 16 waves, one per CU) stages the weight image in
// LDS once; after that single barrier every wave works alone on 16-row tiles dealt round-robin
// over the grid, with its own 18-row X slot in LDS (written and read by that wave only, so no
// further workgroup barrier) and its own register prefetch of the next tile.  Up to 4 waves per
// SIMD keep the MFMA pipe fed while the others run their epilogues, stores and loads.
template <int NB, int KCP, int KS, int TB = 1>
struct C2wCfg {
  static constexpr int KCW = KCP * 16;
  static constexpr int LDX = KCW + 8;          // = c2_ldx: conflict-free b128 operand reads
  static constexpr int NW = NB * 16;
  static constexpr int XROWS = 18;             // 16 rows + the k = 3 halo
  static constexpr int XF4 = XROWS * KCW / 4;  // float4 slots of one X slot
  static constexpr int PF = (XF4 + 63) / 64;   // float4 slots per lane
  static constexpr size_t W_FLOATS = (size_t)KS * NW * LDX;
  static constexpr size_t X_FLOATS = (size_t)XROWS * LDX;
  static constexpr int ET = 1 + 16 * TB;                          // rows of [bias | tail weight]
  static constexpr size_t E_FLOATS = (size_t)NW * ET + 16 * TB;  // bias, tail weight (16 TB x NW), tail bias
  static constexpr size_t lds(int wpg) { return (W_FLOATS + E_FLOATS + (size_t)wpg * X_FLOATS) * 4; }
};

// Per-tile epilogue constants from the workgroup's LDS block Es = [bias (NW) | tail weight (16 TB x NW)
// | tail bias (16 TB)]: bias of this lane's channels, tail weight columns (c2 = l16, and 16 + l16 for
// the second block), tail bias of c2 = 4 lg4 .. (+16).
template <int NB, int TB, int NW, int ET>
__device__ __forceinline__ void c2_tail_consts(const float* Es, int lg4, int l16, bool tail, float (&bias_r)[NB][4],
                                               float (&tw)[NB][4], float (&tw2)[NB][4], f32x4& tb0, f32x4& tb1) {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const float4 b4 = *reinterpret_cast<const float4*>(Es + nb * 16 + 4 * lg4);
    bias_r[nb][0] = b4.x; bias_r[nb][1] = b4.y; bias_r[nb][2] = b4.z; bias_r[nb][3] = b4.w;
    if (tail) {
      const float4 t4 = *reinterpret_cast<const float4*>(Es + NW + l16 * NW + nb * 16 + 4 * lg4);
      tw[nb][0] = t4.x; tw[nb][1] = t4.y; tw[nb][2] = t4.z; tw[nb][3] = t4.w;
      if constexpr (TB > 1) {
        const float4 u4 = *reinterpret_cast<const float4*>(Es + NW + (16 + l16) * NW + nb * 16 + 4 * lg4);
        tw2[nb][0] = u4.x; tw2[nb][1] = u4.y; tw2[nb][2] = u4.z; tw2[nb][3] = u4.w;
      }
    }
  }
  if (tail) {
    const float4 t4 = *reinterpret_cast<const float4*>(Es + ET * NW + 4 * lg4);
    tb0 = f32x4{t4.x, t4.y, t4.z, t4.w};
    if constexpr (TB > 1) {
      const float4 u4 = *reinterpret_cast<const float4*>(Es + ET * NW + 16 + 4 * lg4);
      tb1 = f32x4{u4.x, u4.y, u4.z, u4.w};
    }
  }
}

}  // namespace vqhmm
