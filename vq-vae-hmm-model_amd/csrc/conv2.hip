// Conv1d forward / data-gradient for the small-channel regime of the training
// path (N <= 64 output channels, Kc <= 64 input channels: BASELINE cfg2, cfg4),
// replacing the generic conv_mm_kernel there.
//
//  * Persistent workgroups: the whole (tap, n, c) weight tile is staged in LDS
//    ONCE per workgroup (transposed/flipped for the data gradient) and the
//    workgroup walks row tiles of 4*PB*16 PCL rows with stride gridDim.x.
//  * The next tile's input rows are prefetched into registers (float4 loads,
//    clamped + selected, no branches) while the MFMAs of the current tile run.
//  * The product is computed transposed, Y^T (N x rows) = W (N x 3Kc) @ Xwin^T,
//    so an accumulator fragment holds 4 consecutive channels of one row:
//    epilogue stores are float4, and the fused 1x1 tail (to_logits /
//    to_params, + softmax) consumes the fragments directly as its MFMA B
//    operand (contraction over the fragment's row index), with no LDS round trip.
#include <stdlib.h>

#include "conv2_dev.h"
#include "prof.h"

namespace vqhmm {

// The fused 1x1 tail: one 16-channel block with any outputs, or (C2 <= 32, e.g. to_params at D = 16)
// two blocks without the softmax outputs (q / regimes need the row's channels in one block).
static bool conv2_tail_ok(const ConvArgs& a) {
  return a.tW == nullptr || a.C2 <= 16 || (a.C2 <= 32 && !a.q_out && !a.q_cf && !a.reg_out);
}


// Waves per SIMD the register budget is sized for: the narrow-input layers are
// latency/HBM-bound and their LDS footprint allows 4 workgroups per CU, so they
// are held to 128 VGPRs (ACT / TAIL are template parameters, so a variant only
// keeps the epilogue state it uses); the 64-wide layers are LDS-limited to 2 per CU.
template <int NB, int KCP, bool TAIL>
struct C2Occ {
  static constexpr int W = (KCP <= 2 && !TAIL) ? 4 : 1;
};

template <int NB, int KCP, int KS, int PB, int ACT, bool TAIL>
__global__ __launch_bounds__(256, (C2Occ<NB, KCP, TAIL>::W)) void conv2_kernel(ConvArgs a, int64_t ntiles) {
  using C = C2Cfg<NB, KCP, KS, PB>;
  extern __shared__ float4 smem4[];
  float* Ws = reinterpret_cast<float*>(smem4);  // [KS][NW][LDX]
  float* Xs = Ws + C::W_FLOATS;                 // [XROWS][LDX]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;

  // ---- weights once: Ws[tap][n][c] = Weff(n, c, tap)
  if (a.Wimg) {  // the step's prologue packed them in exactly this layout: float4 copy
    const float4* src = reinterpret_cast<const float4*>(a.Wimg);
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = tid; i < (int)(C::W_FLOATS / 4); i += 256) smem4[i] = src[i];
  } else {
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = tid; i < KS * C::NW * C::KCW; i += 256) {
      const int c = i % C::KCW, n = (i / C::KCW) % C::NW, tap = i / (C::KCW * C::NW);
      float v = 0.f;
      if (n < a.N && c < a.Kc)
        v = a.w_dgrad ? a.W[((int64_t)c * a.N + n) * KS + (KS - 1 - tap)] : a.W[((int64_t)n * a.Kc + c) * KS + tap];
      Ws[(tap * C::NW + n) * C::LDX + c] = v;
    }
  }
  // ---- per-lane epilogue constants
  float bias_r[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int n = nb * 16 + 4 * lg4 + v;
      bias_r[nb][v] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
    }
  constexpr bool tail = TAIL;
  float tw[NB][4];
  f32x4 tb0 = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (TAIL) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int n = nb * 16 + 4 * lg4 + v;
        tw[nb][v] = (l16 < a.C2 && n < a.N) ? a.tW[(int64_t)l16 * a.N + n] : 0.f;
      }
#pragma unroll
    for (int v = 0; v < 4; ++v) tb0[v] = (a.tb && 4 * lg4 + v < a.C2) ? a.tb[4 * lg4 + v] : 0.f;
  }
  const float sc = a.scale ? *a.scale : 1.0f;

  int64_t tile = blockIdx.x;
  float4 pf[C::PF];
#pragma unroll
  for (int k = 0; k < C::PF; ++k) {
    const int s = tid + k * 256;
    pf[k] = x_raw(a, tile * C::BM, s < C::XF4 ? s : 0, C::KCW);
  }
  while (tile < ntiles) {
    const int64_t m0 = tile * C::BM;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < C::PF; ++k) {
      const int s = tid + k * 256;
      if (s < C::XF4) {
        const int row = s / (C::KCW / 4), c = (s - row * (C::KCW / 4)) * 4;
        *reinterpret_cast<float4*>(Xs + row * C::LDX + c) = x_mask(a, m0, s, C::KCW, pf[k]);
      }
    }
    __syncthreads();
    // epilogue operands of THIS tile first (older than the prefetch in the vmcnt order)
    float4 auxv[NB][PB] = {};
    if constexpr (ACT == 2) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int pb = 0; pb < PB; ++pb) {
          const int64_t r = m0 + (wave * PB + pb) * 16 + l16;
          const int n0 = nb * 16 + 4 * lg4;
          const int ldn = ld4(a.N);
          auxv[nb][pb] = *reinterpret_cast<const float4*>(a.aux + (r < a.R ? r : a.R - 1) * ldn + min(n0, ldn - 4));
        }
    }
    const int64_t next = tile + gridDim.x;
    {  // unconditional: see conv2w_kernel
      const int64_t pt = next < ntiles ? next : tile;
#pragma unroll
      for (int k = 0; k < C::PF; ++k) {
        const int s = tid + k * 256;
        pf[k] = x_raw(a, pt * C::BM, s < C::XF4 ? s : 0, C::KCW);
      }
    }
    // ---- MFMA: acc[nb][pb] = Y^T block (16 n x 16 rows)
    f32x4 acc[NB][PB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) acc[nb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
    c2_mfma_tile<NB, PB, KCP, KS, C::LDX, C::NW>(Ws, Xs + (wave * PB) * 16 * C::LDX, lg4, l16, acc, a.pipe);
    conv2_epilogue<NB, PB, ACT>(a, m0, wave, lg4, l16, acc, auxv, bias_r, tw, tb0, sc, tail);
    tile = next;
  }
}


// waves per workgroup the register budget is sized for: 4 per SIMD (128 VGPRs) where that fits
// without spills, 3 (170) for the wide layers
template <int NB, int KCP>
struct C2wOcc {
  static constexpr int MAXW = NB * KCP >= 8 ? 12 : 16;
};

template <int NB, int KCP, int KS, int ACT, int TAIL, bool PK = false>
__global__ __launch_bounds__((64 * C2wOcc<NB, KCP>::MAXW)) void conv2w_kernel(ConvArgs a, int64_t ntiles) {
  constexpr int TBC = TAIL > 1 ? TAIL : 1;  // tail blocks
  using C = C2wCfg<NB, KCP, KS, TBC>;
  extern __shared__ float4 smem4[];
  float* Ws = reinterpret_cast<float*>(smem4);  // [KS][NW][LDX]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwv = blockDim.x >> 6;
  float* Es = Ws + C::W_FLOATS;                       // bias [NW], tail weight [16][NW], tail bias [16]
  float* Xs = Es + C::E_FLOATS + wave * C::X_FLOATS;  // this wave's [XROWS][LDX]
  const int lg4 = lane >> 4, l16 = lane & 15;

  if (a.Wimg) {
    const float4* src = reinterpret_cast<const float4*>(a.Wimg);
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = tid; i < (int)(C::W_FLOATS / 4); i += blockDim.x) smem4[i] = src[i];
  } else {
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = tid; i < KS * C::NW * C::KCW; i += blockDim.x) {
      const int c = i % C::KCW, n = (i / C::KCW) % C::NW, tap = i / (C::KCW * C::NW);
      float v = 0.f;
      if (n < a.N && c < a.Kc)
        v = a.w_dgrad ? a.W[((int64_t)c * a.N + n) * KS + (KS - 1 - tap)] : a.W[((int64_t)n * a.Kc + c) * KS + tap];
      Ws[(tap * C::NW + n) * C::LDX + c] = v;
    }
  }
  // epilogue constants in LDS (read back per tile: registers go to the MFMA loop's prefetch)
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < (int)C::E_FLOATS; i += blockDim.x) {
    float v = 0.f;
    if (i < C::NW) {
      v = (a.bias && i < a.N) ? a.bias[i] : 0.f;
    } else if (i < C::ET * C::NW) {
      const int j = i - C::NW, c2 = j / C::NW, n = j - c2 * C::NW;
      v = (TAIL && c2 < a.C2 && n < a.N) ? a.tW[(int64_t)c2 * a.N + n] : 0.f;
    } else {
      const int c2 = i - C::ET * C::NW;
      v = (TAIL && a.tb && c2 < a.C2) ? a.tb[c2] : 0.f;
    }
    Es[i] = v;
  }
  const float sc = a.scale ? *a.scale : 1.0f;

  // tile = blockIdx.x + gridDim.x * (wave + nwv * k): every workgroup (CU) gets within one tile of
  // the same count, and inside it the extra tiles go to different waves (SIMDs)
  const int64_t stride = (int64_t)gridDim.x * nwv;
  int64_t tile = (int64_t)wave * gridDim.x + blockIdx.x;
  float4 pf[C::PF];
#pragma unroll
  for (int k = 0; k < C::PF; ++k) {
    const int s = lane + k * 64;
    pf[k] = x_raw(a, tile * 16, s < C::XF4 ? s : 0, C::KCW);
  }
  __syncthreads();  // the weights; from here on the waves never wait for each other
  while (tile < ntiles) {
    const int64_t m0 = tile * 16;
#pragma unroll
    for (int k = 0; k < C::PF; ++k) {
      const int s = lane + k * 64;
      if (s < C::XF4) {
        const int row = s / (C::KCW / 4), c = (s - row * (C::KCW / 4)) * 4;
        *reinterpret_cast<float4*>(Xs + row * C::LDX + c) = x_mask(a, m0, s, C::KCW, pf[k]);
      }
    }
    __builtin_amdgcn_wave_barrier();  // LDS ops of a wave run in order; keep the compiler from hoisting reads
    float4 auxv[NB][1] = {};
    if constexpr (ACT == 2) {
      const int64_t r = m0 + l16;
      const int ldn = ld4(a.N);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        auxv[nb][0] = *reinterpret_cast<const float4*>(a.aux + (r < a.R ? r : a.R - 1) * ldn + min(nb * 16 + 4 * lg4, ldn - 4));
    }
    const int64_t next = tile + stride;
    {  // unconditional (a past-the-end tile reads clamped rows, unused): a conditional prefetch makes
       // the compiler's vmcnt accounting assume it may be absent, so the epilogue's wait for the aux
       // loads would also wait for the prefetch
      const int64_t pt = next < ntiles ? next : tile;
#pragma unroll
      for (int k = 0; k < C::PF; ++k) {
        const int s = lane + k * 64;
        pf[k] = x_raw(a, pt * 16, s < C::XF4 ? s : 0, C::KCW);
      }
    }
    f32x4 acc[NB][1];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PK) c2_mfma_pk<NB, C::LDX, C::NW>(Ws, Xs, lg4, l16, a.Kc, acc);
    else c2_mfma_tile<NB, 1, KCP, KS, C::LDX, C::NW>(Ws, Xs, lg4, l16, acc, a.pipe);
    __builtin_amdgcn_wave_barrier();  // the slot's reads are done before the next tile overwrites it
    float bias_r[NB][4], tw[NB][4], tw2[NB][4];
    f32x4 tb0 = f32x4{0.f, 0.f, 0.f, 0.f}, tb1 = tb0;
    c2_tail_consts<NB, TBC, C::NW, C::ET>(Es, lg4, l16, TAIL != 0, bias_r, tw, tw2, tb0, tb1);
    conv2_epilogue<NB, 1, ACT, TBC>(a, m0, 0, lg4, l16, acc, auxv, bias_r, tw, tb0, sc, TAIL, 0, 16, nullptr, 0, tw2,
                                    tb1);
    tile = next;
  }
}

// waves per workgroup cap for the wave-independent conv kernels (VQHMM_CONV_WMAX, A/B; read once)
static int conv_wmax(int dflt) {
  static const int v = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_CONV_WMAX");
    return e ? atoi(e) : 0;
  }();
  return v >= 1 && v < dflt ? v : dflt;
}

// ---------------------------------------------------------------------------------------------
// Fused pair: a k=3 ReLU "front" conv (<= 16 -> Kc channels, Kc <= 64) feeding this k=3 conv
// (enc_conv1 -> enc_conv2 + to_logits, composed dec_conv1 -> dec_conv2 + to_params).  Tiles of 14
// output rows; per tile the wave computes the front conv's 16 rows m0-1 .. m0+14 (one MFMA block
// over 18 input rows in its X1 slot), stores its own rows m0 .. m0+13 to f_out (the backward needs
// them), and writes all 16 into its X slot as this conv's input: the front activation is never
// re-read from HBM and the front launch disappears.  Every front row goes through the unfused
// launch's MFMA sequence and epilogue, so stored and consumed values are the same bits as the
// two-launch path (a halo row is computed by both tiles that touch it, identically).
template <int NB, int TAIL, int FKS, int FKCP = 1>
struct C2fCfg {
  using C = C2wCfg<NB, 4, 3, (TAIL > 1 ? TAIL : 1)>;  // this conv: 33 .. 64 input channels
  using F = C2wCfg<4, FKCP, FKS>;  // front: <= 16 FKCP -> <= 64 channels
  static constexpr int TR = 14;  // output rows per tile
  static constexpr size_t lds(int wpg) {
    return (C::W_FLOATS + C::E_FLOATS + F::W_FLOATS + 64 + (size_t)wpg * (F::X_FLOATS + C::X_FLOATS)) * 4;
  }
};

template <int NB, int TAIL, int FKS, int ACT, bool FPK, int FKCP = 1>
__global__ __launch_bounds__(64 * 12) void conv2f_kernel(ConvArgs a, int64_t ntiles) {
  constexpr int TBC = TAIL > 1 ? TAIL : 1;
  using Q = C2fCfg<NB, TAIL, FKS, FKCP>;
  using C = typename Q::C;
  using F = typename Q::F;
  constexpr int TR = Q::TR;
  extern __shared__ float4 smem4[];
  float* Ws = reinterpret_cast<float*>(smem4);  // this conv's image [3][NW][LDX]
  float* Es = Ws + C::W_FLOATS;                 // bias, tail weight, tail bias
  float* Fs = Es + C::E_FLOATS;                 // front image [3][64][F::LDX]
  float* Fb = Fs + F::W_FLOATS;                 // front bias [64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwv = blockDim.x >> 6;
  float* X1 = Fb + 64 + wave * (F::X_FLOATS + C::X_FLOATS);  // front input rows m0-2 .. m0+15
  float* Xs = X1 + F::X_FLOATS;                                // front output rows m0-1 .. m0+14
  const int lg4 = lane >> 4, l16 = lane & 15;
  stamp_if(a.prof, 0);

  {
    const float4* src = reinterpret_cast<const float4*>(a.Wimg);
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = tid; i < (int)(C::W_FLOATS / 4); i += blockDim.x) smem4[i] = src[i];
    const float4* fsrc = reinterpret_cast<const float4*>(a.f_Wimg);
    float4* fdst = reinterpret_cast<float4*>(Fs);
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = tid; i < (int)(F::W_FLOATS / 4); i += blockDim.x) fdst[i] = fsrc[i];
  }
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < (int)C::E_FLOATS; i += blockDim.x) {
    float v = 0.f;
    if (i < C::NW) {
      v = (a.bias && i < a.N) ? a.bias[i] : 0.f;
    } else if (i < C::ET * C::NW) {
      const int j = i - C::NW, c2 = j / C::NW, n = j - c2 * C::NW;
      v = (TAIL && c2 < a.C2 && n < a.N) ? a.tW[(int64_t)c2 * a.N + n] : 0.f;
    } else {
      const int c2 = i - C::ET * C::NW;
      v = (TAIL && a.tb && c2 < a.C2) ? a.tb[c2] : 0.f;
    }
    Es[i] = v;
  }
  for (int i = tid; i < 64; i += blockDim.x) Fb[i] = (a.f_bias && i < a.Kc) ? a.f_bias[i] : 0.f;
  // the front conv as an ordinary ConvArgs (input = this launch's src)
  ConvArgs fa = a;
  fa.Kc = a.f_Kc; fa.N = a.Kc; fa.out = a.f_out; fa.out_cf = nullptr; fa.scale = a.f_scale; fa.aux = a.f_aux;
  const float sc = a.scale ? *a.scale : 1.0f;
  const float fsc = fa.scale ? *fa.scale : 1.0f;
  const int ldn1 = ld4(fa.N), ldn = ld4(a.N);

  const int64_t stride = (int64_t)gridDim.x * nwv;
  int64_t tile = (int64_t)wave * gridDim.x + blockIdx.x;
  float4 pf[F::PF];
#pragma unroll
  for (int k = 0; k < F::PF; ++k) {
    const int s = lane + k * 64;
    pf[k] = x_raw(fa, tile * TR - 1, s < F::XF4 ? s : 0, F::KCW);
  }
  __syncthreads();  // weights; from here on the waves never wait for each other
  stamp_if(a.prof, 1);
  int ntl = 0;
  while (tile < ntiles) {
    const int64_t m0 = tile * TR;
    // ReLU masks of both epilogues (ACT = 2), older than the prefetch in the vmcnt order
    float4 aux1[4][1] = {}, auxv[NB][1] = {};
    if constexpr (ACT == 2) {
      const int64_t r1 = m0 - 1 + l16, r = m0 + l16;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        aux1[nb][0] = *reinterpret_cast<const float4*>(fa.aux + (r1 < 0 ? 0 : (r1 < a.R ? r1 : a.R - 1)) * ldn1 +
                                                       min(nb * 16 + 4 * lg4, ldn1 - 4));
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        auxv[nb][0] = *reinterpret_cast<const float4*>(a.aux + (r < a.R ? r : a.R - 1) * ldn + min(nb * 16 + 4 * lg4, ldn - 4));
    }
#pragma unroll
    for (int k = 0; k < F::PF; ++k) {
      const int s = lane + k * 64;
      if (s < F::XF4) {
        const int row = s / (F::KCW / 4), c = (s - row * (F::KCW / 4)) * 4;
        *reinterpret_cast<float4*>(X1 + row * F::LDX + c) = x_mask(fa, m0 - 1, s, F::KCW, pf[k]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    const int64_t next = tile + stride;
    {  // unconditional prefetch, as in conv2w_kernel
      const int64_t pt = next < ntiles ? next : tile;
#pragma unroll
      for (int k = 0; k < F::PF; ++k) {
        const int s = lane + k * 64;
        pf[k] = x_raw(fa, pt * TR - 1, s < F::XF4 ? s : 0, F::KCW);
      }
    }
    // ---- front conv: rows m0-1 .. m0+14
    f32x4 acc1[4][1];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc1[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (FPK) c2_mfma_pk<4, F::LDX, F::NW>(Fs, X1, lg4, l16, a.f_Kc, acc1);  // = the unfused front's
    else c2_mfma_tile<4, 1, FKCP, FKS, F::LDX, F::NW>(Fs, X1, lg4, l16, acc1, a.pipe);
    {
      float b1[4][4], tw0[4][4] = {};
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float4 b4 = *reinterpret_cast<const float4*>(Fb + nb * 16 + 4 * lg4);
        b1[nb][0] = b4.x; b1[nb][1] = b4.y; b1[nb][2] = b4.z; b1[nb][3] = b4.w;
      }
      conv2_epilogue<4, 1, ACT>(fa, m0 - 1, 0, lg4, l16, acc1, aux1, b1, tw0, f32x4{0.f, 0.f, 0.f, 0.f}, fsc, false,
                                1, TR + 1);
    }
    // activated rows (0 outside sequences) -> this conv's input slot
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) *reinterpret_cast<f32x4*>(Xs + l16 * C::LDX + nb * 16 + 4 * lg4) = acc1[nb][0];
    __builtin_amdgcn_wave_barrier();
    // ---- this conv: rows m0 .. m0+13 (block rows 14, 15 are the next tile's: not stored)
    f32x4 acc[NB][1];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    c2_mfma_tile<NB, 1, 4, 3, C::LDX, C::NW>(Ws, Xs, lg4, l16, acc, a.pipe);
    __builtin_amdgcn_wave_barrier();  // the slots' reads are done before the next tile overwrites them
    float bias_r[NB][4], tw[NB][4], tw2[NB][4];
    f32x4 tb0 = f32x4{0.f, 0.f, 0.f, 0.f}, tb1 = tb0;
    c2_tail_consts<NB, TBC, C::NW, C::ET>(Es, lg4, l16, TAIL != 0, bias_r, tw, tw2, tb0, tb1);
    conv2_epilogue<NB, 1, ACT, TBC>(a, m0, 0, lg4, l16, acc, auxv, bias_r, tw, tb0, sc, TAIL, 0, TR, nullptr, 0, tw2,
                                    tb1);
    tile = next;
    if (ntl++ == 0) stamp_if(a.prof, 2);
  }
  if (a.prof) {
    __syncthreads();
    stamp_if(true, 7);
    if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 8] = (unsigned long long)ntl;
  }
}

template <int NB, int TAIL, int FKS, int ACT, int FKCP = 1>
static int launch_c2f(const ConvArgs& a, hipStream_t s) {
  using Q = C2fCfg<NB, TAIL, FKS, FKCP>;
  ConvArgs ap = a;
  ap.pipe = 1;
  static const int prof = prof_env("VQHMM_CONV_PROF");
  ap.prof = prof;
  const int64_t ntiles = cdiv(a.R, Q::TR);
  int wmax = conv_wmax(12);
  while (wmax > 1 && Q::lds(wmax) > 160 * 1024) --wmax;
  if (Q::lds(wmax) > 160 * 1024) return VQHMM_EUNSUPPORTED;
  const int64_t want = cdiv(ntiles, 256);
  const int wpg = (int)(want < wmax ? (want > 0 ? want : 1) : wmax);
  const int64_t grid = cdiv(ntiles, wpg) < 256 ? cdiv(ntiles, wpg) : 256;
  bool pk = false;
  if constexpr (FKS == 3) pk = 3 * a.f_Kc <= 16;  // packed front taps, as launch_c2w runs the unfused front
  if constexpr (FKS == 3) {
    if (pk) {
      conv2f_kernel<NB, TAIL, FKS, ACT, true><<<(unsigned)grid, 64 * wpg, Q::lds(wpg), s>>>(ap, ntiles);
      VQHMM_LAUNCH_CHECK();
      return VQHMM_OK;
    }
  }
  conv2f_kernel<NB, TAIL, FKS, ACT, false, FKCP><<<(unsigned)grid, 64 * wpg, Q::lds(wpg), s>>>(ap, ntiles);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

bool conv2_fused_supported(const ConvArgs& a) {
  const bool relu_pair = a.act == 1 && a.f_act == 1 && a.f_ks == 3;                        // forward
  const bool mask_pair = a.act == 2 && a.f_act == 2 && a.f_ks == 1 && a.aux && a.f_aux && !a.tW;  // data grad
  // front input channels: <= 16 (one k-block), or <= 32 for the 1x1 data-gradient front (to_params at D = 16)
  return a.f_Wimg && a.Wimg && a.f_out && !a.src_cf && a.ks == 3 && (relu_pair || mask_pair) && a.f_Kc >= 1 &&
         (a.f_Kc <= 16 || (mask_pair && a.f_Kc <= 32)) && a.Kc > 32 && a.Kc <= 64 && a.N <= 64 && conv2_tail_ok(a) &&
         !a.out_cf;
}

int launch_conv2_fused(const ConvArgs& a, hipStream_t s) {
  if (!conv2_fused_supported(a)) return VQHMM_EUNSUPPORTED;
  if (a.R == 0) return VQHMM_OK;
  if (a.act == 2) {
    if (a.f_Kc > 16)
      return a.N <= 64 && a.N > 32 ? launch_c2f<4, 0, 1, 2, 2>(a, s)
             : a.N > 16 ? launch_c2f<2, 0, 1, 2, 2>(a, s) : launch_c2f<1, 0, 1, 2, 2>(a, s);
    return a.N <= 64 && a.N > 32 ? launch_c2f<4, 0, 1, 2>(a, s)
           : a.N > 16 ? launch_c2f<2, 0, 1, 2>(a, s) : launch_c2f<1, 0, 1, 2>(a, s);
  }
  const int tail = a.tW == nullptr ? 0 : a.C2 > 16 ? 2 : 1;
  if (a.N <= 16)
    return tail == 2 ? launch_c2f<1, 2, 3, 1>(a, s) : tail ? launch_c2f<1, 1, 3, 1>(a, s) : launch_c2f<1, 0, 3, 1>(a, s);
  if (a.N <= 32)
    return tail == 2 ? launch_c2f<2, 2, 3, 1>(a, s) : tail ? launch_c2f<2, 1, 3, 1>(a, s) : launch_c2f<2, 0, 3, 1>(a, s);
  return tail == 2 ? launch_c2f<4, 2, 3, 1>(a, s) : tail ? launch_c2f<4, 1, 3, 1>(a, s) : launch_c2f<4, 0, 3, 1>(a, s);
}

// ---------------------------------------------------------------------------------------------
// Fused backward pair: dec_conv1 dgrad (H -> K, k = 3) whose epilogue runs the softmax backward and
// to_logits' masked data gradient (ACT = 3 with lb_dh: dh2, H2 channels), feeding enc_conv2's
// masked data gradient (H2 -> H, k = 3).  14-row tiles as conv2f_kernel: the front computes rows
// m0-1 .. m0+14, stores its own rows' dqd / dlog / dh2 and writes all 16 dh2 rows into the X slot;
// dh2 is never re-read from HBM.  Same arithmetic per row as the two launches (bit-identical).
template <int NB, int KCP>
struct C2gCfg {
  using C = C2wCfg<NB, KCP, 3>;  // enc_conv2 dgrad: H2 -> H
  using F = C2wCfg<1, 4, 3>;     // dec_conv1 dgrad: H (33 .. 64) -> K (<= 4)
  static constexpr int TR = 14;
  static constexpr size_t lds(int wpg) {
    return (C::W_FLOATS + F::W_FLOATS + (size_t)wpg * (F::X_FLOATS + C::X_FLOATS)) * 4;
  }
};

template <int NB, int KCP>
__global__ __launch_bounds__(64 * 12) void conv2g_kernel(ConvArgs a, ConvArgs f, int64_t ntiles) {
  using Q = C2gCfg<NB, KCP>;
  using C = typename Q::C;
  using F = typename Q::F;
  constexpr int TR = Q::TR;
  extern __shared__ float4 smem4[];
  float* Ws = reinterpret_cast<float*>(smem4);  // enc_conv2 dgrad image
  float* Fs = Ws + C::W_FLOATS;                 // dec_conv1 dgrad image
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwv = blockDim.x >> 6;
  float* X1 = Fs + F::W_FLOATS + wave * (F::X_FLOATS + C::X_FLOATS);  // dg1 rows m0-2 .. m0+15
  float* Xs = X1 + F::X_FLOATS;                                         // dh2 rows m0-1 .. m0+14
  const int lg4 = lane >> 4, l16 = lane & 15;
  {
    const float4* src = reinterpret_cast<const float4*>(a.Wimg);
#pragma unroll 8
    for (int i = tid; i < (int)(C::W_FLOATS / 4); i += blockDim.x) smem4[i] = src[i];
    const float4* fsrc = reinterpret_cast<const float4*>(f.Wimg);
    float4* fdst = reinterpret_cast<float4*>(Fs);
#pragma unroll 8
    for (int i = tid; i < (int)(F::W_FLOATS / 4); i += blockDim.x) fdst[i] = fsrc[i];
  }
  const float sc = a.scale ? *a.scale : 1.0f, fsc = f.scale ? *f.scale : 1.0f;
  const int ldn = ld4(a.N);
  const int64_t stride = (int64_t)gridDim.x * nwv;
  int64_t tile = (int64_t)wave * gridDim.x + blockIdx.x;
  float4 pf[F::PF];
#pragma unroll
  for (int k = 0; k < F::PF; ++k) {
    const int s = lane + k * 64;
    pf[k] = x_raw(f, tile * TR - 1, s < F::XF4 ? s : 0, F::KCW);
  }
  __syncthreads();  // weights; from here on the waves never wait for each other
  const float zb1[1][4] = {}, zbN[NB][4] = {}, tw1[1][4] = {}, twN[NB][4] = {};
  const float4 aux1[1][1] = {};
  while (tile < ntiles) {
    const int64_t m0 = tile * TR;
    float4 auxv[NB][1];
    {
      const int64_t r = m0 + l16;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        auxv[nb][0] = *reinterpret_cast<const float4*>(a.aux + (r < a.R ? r : a.R - 1) * ldn + min(nb * 16 + 4 * lg4, ldn - 4));
    }
#pragma unroll
    for (int k = 0; k < F::PF; ++k) {
      const int s = lane + k * 64;
      if (s < F::XF4) {
        const int row = s / (F::KCW / 4), c = (s - row * (F::KCW / 4)) * 4;
        *reinterpret_cast<float4*>(X1 + row * F::LDX + c) = x_mask(f, m0 - 1, s, F::KCW, pf[k]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    const int64_t next = tile + stride;
    {
      const int64_t pt = next < ntiles ? next : tile;
#pragma unroll
      for (int k = 0; k < F::PF; ++k) {
        const int s = lane + k * 64;
        pf[k] = x_raw(f, pt * TR - 1, s < F::XF4 ? s : 0, F::KCW);
      }
    }
    f32x4 acc1[1][1] = {{f32x4{0.f, 0.f, 0.f, 0.f}}};
    c2_mfma_tile<1, 1, 4, 3, F::LDX, F::NW>(Fs, X1, lg4, l16, acc1, 1);
    conv2_epilogue<1, 1, 3>(f, m0 - 1, 0, lg4, l16, acc1, aux1, zb1, tw1, f32x4{0.f, 0.f, 0.f, 0.f}, fsc, false, 1,
                            TR + 1, Xs, C::LDX);
    __builtin_amdgcn_wave_barrier();
    f32x4 acc[NB][1];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    c2_mfma_tile<NB, 1, KCP, 3, C::LDX, C::NW>(Ws, Xs, lg4, l16, acc, 1);
    __builtin_amdgcn_wave_barrier();  // the slots' reads are done before the next tile overwrites them
    conv2_epilogue<NB, 1, 2>(a, m0, 0, lg4, l16, acc, auxv, zbN, twN, f32x4{0.f, 0.f, 0.f, 0.f}, sc, false, 0, TR);
    tile = next;
  }
}

template <int NB, int KCP>
static int launch_c2g(const ConvArgs& a, const ConvArgs& f, hipStream_t s) {
  using Q = C2gCfg<NB, KCP>;
  const int64_t ntiles = cdiv(a.R, Q::TR);
  int wmax = conv_wmax(12);  // 3 waves / SIMD (a few bytes of spill) measured faster than 2 without (cfg2 72 vs 78 us)
  while (wmax > 1 && Q::lds(wmax) > 160 * 1024) --wmax;
  if (Q::lds(wmax) > 160 * 1024) return VQHMM_EUNSUPPORTED;
  const int64_t want = cdiv(ntiles, 256);
  const int wpg = (int)(want < wmax ? (want > 0 ? want : 1) : wmax);
  const int64_t grid = cdiv(ntiles, wpg) < 256 ? cdiv(ntiles, wpg) : 256;
  conv2g_kernel<NB, KCP><<<(unsigned)grid, 64 * wpg, Q::lds(wpg), s>>>(a, f, ntiles);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// a: enc_conv2 dgrad (act 2), f: dec_conv1 dgrad with the fused logits backward + to_logits dgrad
bool conv2_bwd_pair_supported(const ConvArgs& a, const ConvArgs& f) {
  const int L = ld4(f.lb_C);
  const int kcw = a.Kc <= 16 ? 16 : a.Kc <= 32 ? 32 : 64;
  return a.Wimg && f.Wimg && f.act == 3 && f.lb_dh && f.N <= 4 && f.Kc > 32 && f.Kc <= 64 && f.ks == 3 &&
         a.ks == 3 && a.act == 2 && a.aux && a.N <= 64 && a.N > 32 && a.Kc == f.lb_C && L == kcw && !a.src_cf &&
         !f.src_cf && !a.out_cf && !f.out_cf && !a.tW && a.R == f.R;
}

int launch_conv2_bwd_pair(const ConvArgs& a, const ConvArgs& f, hipStream_t s) {
  if (!conv2_bwd_pair_supported(a, f)) return VQHMM_EUNSUPPORTED;
  if (a.R == 0) return VQHMM_OK;
  if (a.Kc <= 16) return launch_c2g<4, 1>(a, f, s);
  if (a.Kc <= 32) return launch_c2g<4, 2>(a, f, s);
  return launch_c2g<4, 4>(a, f, s);
}

// Kernel choice: VQHMM_CONV=wg | wave forces one (A/B), else the wave kernel below
// VQHMM_CONV_WAVE_ROWS rows (default: always; it measured equal or faster at B = 128 .. 1024)
// and the workgroup-tile kernel above; VQHMM_CONV_PIPE=0
// turns the operand pipelining off (A/B).  Read once.
static int env_int(const char* e, int dflt) { return e ? atoi(e) : dflt; }
static bool conv2_wave_mode(int64_t R) {
  static const int force = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_CONV");
    return !e ? 0 : (e[0] == 'w' && e[1] == 'g') ? 1 : (e[0] == 'w' && e[1] == 'a') ? 2 : 0;
  }();
  static const int64_t rows = env_int(VQHMM_PROF_ENV("VQHMM_CONV_WAVE_ROWS"), 1 << 30);
  return force == 2 || (force == 0 && R < rows);
}
static bool conv2_pipe() {
  static const bool v = env_int(VQHMM_PROF_ENV("VQHMM_CONV_PIPE"), 1) != 0;
  return v;
}

template <int NB, int KCP, int KS, int ACT, int TAIL>
static int launch_c2w(const ConvArgs& a, hipStream_t s) {
  using C = C2wCfg<NB, KCP, KS, (TAIL > 1 ? TAIL : 1)>;
  const int64_t ntiles = cdiv(a.R, 16);
  int wmax = conv_wmax(C2wOcc<NB, KCP>::MAXW);
  while (wmax > 1 && C::lds(wmax) > 160 * 1024) --wmax;
  if (C::lds(wmax) > 160 * 1024) return VQHMM_EUNSUPPORTED;
  // one workgroup per CU: as many waves as it takes to give every CU work, up to wmax
  const int64_t want = cdiv(ntiles, 256);
  const int wpg = (int)(want < wmax ? (want > 0 ? want : 1) : wmax);
  const int64_t grid = cdiv(ntiles, wpg) < 256 ? cdiv(ntiles, wpg) : 256;
  if constexpr (KCP == 1 && KS == 3) {
    if (3 * a.Kc <= 16) {  // packed taps (c2_mfma_pk)
      conv2w_kernel<NB, KCP, KS, ACT, TAIL, true><<<(unsigned)grid, 64 * wpg, C::lds(wpg), s>>>(a, ntiles);
      VQHMM_LAUNCH_CHECK();
      return VQHMM_OK;
    }
  }
  conv2w_kernel<NB, KCP, KS, ACT, TAIL><<<(unsigned)grid, 64 * wpg, C::lds(wpg), s>>>(a, ntiles);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

bool conv2_supported(const ConvArgs& a) { return !a.src_cf && a.N <= 64 && a.Kc <= 64 && conv2_tail_ok(a); }

template <int NB, int KCP, int KS, int PB, int ACT, int TAIL>
static int launch_c2v(const ConvArgs& a, hipStream_t s) {
  ConvArgs ap = a;
  ap.pipe = conv2_pipe();
  if (conv2_wave_mode(a.R)) return launch_c2w<NB, KCP, KS, ACT, TAIL>(ap, s);
  if constexpr (TAIL > 1) return VQHMM_EUNSUPPORTED;  // the workgroup-tile A/B kernel: one tail block
  using C = C2Cfg<NB, KCP, KS, PB>;
  const int64_t ntiles = cdiv(a.R, C::BM);
  int per_cu = (int)((160 * 1024) / C::LDS);
  if (per_cu < 1) return VQHMM_EUNSUPPORTED;
  if (per_cu > 4) per_cu = 4;
  const int64_t grid = ntiles < 256LL * per_cu ? ntiles : 256LL * per_cu;
  conv2_kernel<NB, KCP, KS, PB, ACT, (TAIL != 0)><<<(unsigned)grid, 256, C::LDS, s>>>(ap, ntiles);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// epilogue variants in use: forward ReLU (+ fused 1x1 tail on k=3), dgrad with
// the producer's ReLU mask, plain dgrad
template <int NB, int KCP, int KS, int PB>
static int launch_c2p(const ConvArgs& a, hipStream_t s) {
  const bool tail = a.tW != nullptr;
  if (tail) {
    if constexpr (KS == 3) {
      if (a.act == 1)
        return a.C2 > 16 ? launch_c2v<NB, KCP, KS, PB, 1, 2>(a, s) : launch_c2v<NB, KCP, KS, PB, 1, 1>(a, s);
    }
    return VQHMM_EUNSUPPORTED;
  }
  if (a.act == 4) {  // K <= 8 softmax backward
    if constexpr (NB == 1 && KS == 3) return launch_c2v<NB, KCP, KS, PB, 4, 0>(a, s);
    return VQHMM_EUNSUPPORTED;
  }
  if (a.act == 3) {
    if constexpr (NB == 1 && KS == 3) return launch_c2v<NB, KCP, KS, PB, 3, 0>(a, s);
    return VQHMM_EUNSUPPORTED;
  }
  if (a.act == 2) return launch_c2v<NB, KCP, KS, PB, 2, 0>(a, s);
  if (a.act == 1) return launch_c2v<NB, KCP, KS, PB, 1, 0>(a, s);
  return launch_c2v<NB, KCP, KS, PB, 0, 0>(a, s);
}

// rows per tile = 64*PB; PB = 1 (measured best: it halves the X tile so more
// workgroups fit per CU)
template <int NB, int KCP, int KS>
static int launch_c2(const ConvArgs& a, hipStream_t s) {
  return launch_c2p<NB, KCP, KS, 1>(a, s);
}

template <int NB, int KS>
static int launch_c2_k(const ConvArgs& a, hipStream_t s) {
  if (a.Kc <= 16) return launch_c2<NB, 1, KS>(a, s);
  if (a.Kc <= 32) return launch_c2<NB, 2, KS>(a, s);
  return launch_c2<NB, 4, KS>(a, s);
}

template <int KS>
static int launch_c2_n(const ConvArgs& a, hipStream_t s) {
  if (a.N <= 16) return launch_c2_k<1, KS>(a, s);
  if (a.N <= 32) return launch_c2_k<2, KS>(a, s);
  return launch_c2_k<4, KS>(a, s);
}

int launch_conv2(const ConvArgs& a, hipStream_t s) {
  if (a.R == 0) return VQHMM_OK;
  return a.ks == 3 ? launch_c2_n<3>(a, s) : launch_c2_n<1>(a, s);
}

int conv2_prof_copy(uint64_t* out, int64_t n) { return prof_copy(out, n); }

}  // namespace vqhmm
