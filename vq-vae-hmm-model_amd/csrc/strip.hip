// Strip kernels: several convolution layers of the training step in ONE launch, the activations
// between the layers kept in LDS (VQ_VAE_HMM_fixed.py:38-41 Encoder.forward, :80-90 Decoder.forward).
//
// A strip is a window of ST_WIN = 128 consecutive PCL rows whose middle ST_OWN = 122 rows it owns.
// Each layer is computed on the whole window (one 16-row MFMA block per wave, 8 waves), so a k = 3
// layer's output is exact one row further inside the window than its input; the forward chain
//   x -> enc_conv1 -> enc_conv2 (+ to_logits, softmax) -> composed dec_conv1 -> dec_conv2 (+ to_params)
// has four k = 3 layers and an LDS input of ST_WIN + 2 rows, so rows >= ST_HALO = 3 from the window
// edges are exact at the end: the strip stores exactly those (owned rows tile [0, R) without overlap).
// No workgroup ever waits for another; the 2.5% of recomputed rows replace four launches' fixed
// costs (weight staging, the first tile's latency, the tail) with one, which is what bounds the
// step at the strong-scaling shard sizes (B = 128 per GPU).
//
// Every row goes through the fused-pair launches' MFMA sequences and epilogue (conv2_dev.h), so
// the stored activations are the same bits as the conv2f path (tests: strip = pair launches).
#include "vqhmm.h"

#include <stddef.h>
#include <stdlib.h>

#include "conv2_dev.h"

namespace vqhmm {

namespace {
constexpr int ST_WIN = 128;                    // window rows: 8 MFMA row blocks, one per wave
constexpr int ST_HALO = 3;                     // recomputed rows on each side
constexpr int ST_OWN = ST_WIN - 2 * ST_HALO;   // rows a strip stores
constexpr int ST_SR = ST_WIN + 2;              // LDS rows of a layer input (the k = 3 halo)
constexpr int ST_XLD = 8;                      // row stride of the narrow buffers (x, q)
constexpr int ST_LDW = 72;                     // c2_ldx(64): 64-channel buffers and weight images
constexpr int ST_LDF = 24;                     // c2_ldx(<= 16): the narrow layers' weight images

// profiling builds (VQHMM_STRIP_PROF=1, read once): s_memrealtime stamps of workgroup w's phases in
// g_prof[w * 16 + k] (vqhmm_debug_prof); results unchanged
__device__ unsigned long long g_prof[256 * 16];
template <bool PROF>
__device__ __forceinline__ void stamp(int k) {
  if constexpr (PROF) {
    if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int NB2>
struct StripFwdLds {
  static constexpr int NW2 = 16 * NB2;
  float We2[3 * NW2 * ST_LDW];  // enc_conv2 image (the prologue's, [tap][n][c])
  float Wd2[3 * 64 * ST_LDW];   // dec_conv2 image
  float Ee2[NW2 * 17 + 16];     // enc_conv2 bias | to_logits weight | bias (c2_tail_consts layout)
  float Ed2[64 * 17 + 16];      // dec_conv2 bias | to_params weight | bias
  float bf[2][64];              // enc_conv1 / composed dec_conv1 bias
  float XA[ST_SR * ST_XLD];     // x rows, then q rows
  float XB[ST_SR * ST_LDW];     // h1 rows, then g1 rows
};

// A packed-tap front conv's weights as c2_mfma_pk gathers them from its image, held in registers
// for the whole launch: w[nb][e] = image value of k-column 4 lg4 + e, output channel nb*16 + l16.
__device__ __forceinline__ void pk_weights(const float* img, int C, int lg4, int l16, float (&w)[4][4]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = 4 * lg4 + e;
    const bool in = k < 3 * C;
    const int tap = in ? k / C : 0, c = in ? k - tap * C : 15;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) w[nb][e] = img[(tap * 64 + nb * 16 + l16) * ST_LDF + c];
  }
}

// c2_mfma_pk with register weights and ST_XLD-stride input rows: the same MFMA sequence (columns
// past 3C multiply the image's zero pad column by 0, as c2_mfma_pk's zero X column does)
__device__ __forceinline__ void pk_mfma(const float (&w)[4][4], const float* Xw, int C, int lg4, int l16,
                                        f32x4 (&acc)[4][1]) {
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
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[nb][0] = mfma16x16x4(w[nb][e], b[e], acc[nb][0]);
}

// element i of a conv2w-style [bias (NW) | tail weight (16 x NW) | tail bias (16)] block (conv2w_kernel's Es)
template <int NW>
__device__ __forceinline__ float es_val(const ConvArgs& a, int i) {
  if (i < NW) return (a.bias && i < a.N) ? a.bias[i] : 0.f;
  if (i < 17 * NW) {
    const int j = i - NW, c2 = j / NW, n = j - c2 * NW;
    return (c2 < a.C2 && n < a.N) ? a.tW[(int64_t)c2 * a.N + n] : 0.f;
  }
  const int c2 = i - 17 * NW;
  return (a.tb && c2 < a.C2) ? a.tb[c2] : 0.f;
}

// a front conv's epilogue (bias, ReLU, pad rows 0; owned rows stored) and its rows into the XB slot
__device__ __forceinline__ void front_out(const ConvArgs& a, int64_t rb, int lg4, int l16, f32x4 (&acc)[4][1],
                                          const float* bias, int rlo, int rhi, float* xb) {
  float b1[4][4], tw0[4][4] = {};
  float4 aux[4][1] = {};
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const float4 b4 = *reinterpret_cast<const float4*>(bias + nb * 16 + 4 * lg4);
    b1[nb][0] = b4.x; b1[nb][1] = b4.y; b1[nb][2] = b4.z; b1[nb][3] = b4.w;
  }
  conv2_epilogue<4, 1, 1>(a, rb, 0, lg4, l16, acc, aux, b1, tw0, f32x4{0.f, 0.f, 0.f, 0.f}, 1.0f, false, rlo, rhi);
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) *reinterpret_cast<f32x4*>(xb + l16 * ST_LDW + nb * 16 + 4 * lg4) = acc[nb][0];
}
}  // namespace

// e1 enc_conv1 (packed taps), e2 enc_conv2 + to_logits + softmax, d1 composed dec_conv1 (packed
// taps), d2 dec_conv2 + to_params: the four ConvArgs of the pair launches (outputs, images, biases).
template <int NB2, bool PROF>
__global__ __launch_bounds__(512) void strip_fwd_kernel(ConvArgs e1, ConvArgs e2, ConvArgs d1, ConvArgs d2,
                                                        int64_t nstrip) {
  using S = StripFwdLds<NB2>;
  constexpr int NW2 = S::NW2;
  extern __shared__ float4 smem4[];
  S& sh = *reinterpret_cast<S*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lg4 = lane >> 4, l16 = lane & 15;
  const int64_t R = e1.R;
  const int ldx = ld4(e1.Kc);  // x row stride (<= 8)

  // x rows of the window at s0: thread i < 2 ST_SR holds float4 i % 2 of LDS row i / 2 (PCL row
  // s0 - 1 + i / 2); the load is unconditional (clamped), the mask applied when it is stored
  auto load_x = [&](int64_t s0) {
    const int row = tid >> 1, h = 4 * (tid & 1);
    int64_t r = s0 - 1 + row;
    r = r < 0 ? 0 : (r >= R ? R - 1 : r);
    return *reinterpret_cast<const float4*>(e1.src + r * ldx + (h < ldx ? h : 0));
  };
  auto store_x = [&](int64_t s0, float4 v) {
    if (tid < 2 * ST_SR) {
      const int row = tid >> 1, h = 4 * (tid & 1);
      const int64_t r = s0 - 1 + row;
      const bool ok = r >= 0 && r < R && h < ldx;
      *reinterpret_cast<float4*>(sh.XA + row * ST_XLD + h) = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  stamp<PROF>(0);
  int64_t s = blockIdx.x;
  float4 px = load_x(s * ST_OWN - ST_HALO);

  // ---- once: epilogue constants, front biases and front weights into registers; then the two
  // 64-wide images by LDS DMA, issued last so that waiting for the register loads never waits for
  // them: they stay in flight through x -> LDS and enc_conv1 (waited for before enc_conv2)
  constexpr int NE = NW2 * 17 + 16, ND = 64 * 17 + 16, NC = NE + ND + 128;  // sh.Ee2 | sh.Ed2 | sh.bf
  constexpr int NCJ = (NC + 511) / 512;
  float cv[NCJ];
#pragma unroll
  for (int j = 0; j < NCJ; ++j) {
    const int i = tid + 512 * j;
    float v = 0.f;
    if (i < NE) {
      v = es_val<NW2>(e2, i);
    } else if (i < NE + ND) {
      v = es_val<64>(d2, i - NE);
    } else if (i < NC) {
      const int k = i - NE - ND, n = k & 63;
      const ConvArgs& f = k < 64 ? e1 : d1;
      v = (f.bias && n < f.N) ? f.bias[n] : 0.f;
    }
    cv[j] = v;
  }
  float wE[4][4], wD[4][4];
  pk_weights(e1.Wimg, e1.Kc, lg4, l16, wE);
  pk_weights(d1.Wimg, d1.Kc, lg4, l16, wD);
  {
    constexpr int N1 = 3 * NW2 * ST_LDW / 4, N2 = 3 * 64 * ST_LDW / 4;  // float4s of each image
    constexpr int C1 = (N1 + 63) / 64, C2 = (N2 + 63) / 64;              // 1 KB chunks (one per wave instruction)
    for (int c = wave; c < C1 + C2; c += 8) {
      const bool first = c < C1;
      const int cc = first ? c : c - C1;
      const int i = cc * 64 + lane;
      const float* src = first ? e2.Wimg : d2.Wimg;
      float* dst = (first ? sh.We2 : sh.Wd2) + cc * 256;
      if (i < (first ? N1 : N2))
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(src) + 4 * i,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  }
  static_assert(offsetof(S, Ed2) == offsetof(S, Ee2) + NE * 4 && offsetof(S, bf) == offsetof(S, Ed2) + ND * 4,
                "constant blocks must be contiguous");
#pragma unroll
  for (int j = 0; j < NCJ; ++j)
    if (tid + 512 * j < NC) sh.Ee2[tid + 512 * j] = cv[j];
  for (int i = tid; i < 2 * ST_LDW; i += 512) sh.XB[(i < ST_LDW ? 0 : (ST_SR - 1) * ST_LDW) + i % ST_LDW] = 0.f;
  lds_barrier();  // LDS only: the image DMA stays in flight
  stamp<PROF>(1);
  int it = 0;  // profiling: the first strip's phases

  // rows of this wave's block that the strip owns
  const int rlo = max(0, ST_HALO - 16 * wave), rhi = min(16, ST_HALO + ST_OWN - 16 * wave);
  for (; s < nstrip; s += gridDim.x) {
    const int64_t s0 = s * ST_OWN - ST_HALO;  // PCL row of window row 0
    const int64_t rb = s0 + 16 * wave;        // PCL row of this wave's block row 0
    store_x(s0, px);
    lds_barrier();
    if (it == 0) stamp<PROF>(2);
    {
      const int64_t nx = s + gridDim.x;
      px = load_x((nx < nstrip ? nx : s) * ST_OWN - ST_HALO);  // the next strip's x, in flight
    }
    // ---- enc_conv1 + ReLU: x (XA) -> h1 (XB, h1e)
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      pk_mfma(wE, sh.XA + 16 * wave * ST_XLD, e1.Kc, lg4, l16, acc);
      front_out(e1, rb, lg4, l16, acc, sh.bf[0], rlo, rhi, sh.XB + (16 * wave + 1) * ST_LDW);
    }
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the image DMA (first strip)
    lds_barrier();
    if (it == 0) stamp<PROF>(3);
    // ---- enc_conv2 + ReLU (h2e) + to_logits (logits) + softmax (q, and q -> XA)
    {
      f32x4 acc[NB2][1];
#pragma unroll
      for (int nb = 0; nb < NB2; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<NB2, 1, 4, 3, ST_LDW, NW2>(sh.We2, sh.XB + 16 * wave * ST_LDW, lg4, l16, acc, true);
      float bias_r[NB2][4], tw[NB2][4], tw2[NB2][4];
      f32x4 tb0 = f32x4{0.f, 0.f, 0.f, 0.f}, tb1 = tb0;
      c2_tail_consts<NB2, 1, NW2, 17>(sh.Ee2, lg4, l16, true, bias_r, tw, tw2, tb0, tb1);
      float4 aux[NB2][1] = {};
      conv2_epilogue<NB2, 1, 1, 1>(e2, rb, 0, lg4, l16, acc, aux, bias_r, tw, tb0, 1.0f, true, rlo, rhi, nullptr, 0,
                                   tw2, tb1, sh.XA + (16 * wave + 1) * ST_XLD, ST_XLD);
    }
    lds_barrier();
    if (it == 0) stamp<PROF>(4);
    // ---- composed dec_conv1 + ReLU: q (XA) -> g1 (XB, g1)
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      pk_mfma(wD, sh.XA + 16 * wave * ST_XLD, d1.Kc, lg4, l16, acc);
      front_out(d1, rb, lg4, l16, acc, sh.bf[1], rlo, rhi, sh.XB + (16 * wave + 1) * ST_LDW);
    }
    lds_barrier();
    if (it == 0) stamp<PROF>(5);
    // ---- dec_conv2 + ReLU (g2) + to_params (par).  No barrier after it: the next strip's x goes
    // to XA (last read before the barrier above), and its barrier orders XB's next writes.
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2_mfma_tile<4, 1, 4, 3, ST_LDW, 64>(sh.Wd2, sh.XB + 16 * wave * ST_LDW, lg4, l16, acc, true);
      float bias_r[4][4], tw[4][4], tw2[4][4];
      f32x4 tb0 = f32x4{0.f, 0.f, 0.f, 0.f}, tb1 = tb0;
      c2_tail_consts<4, 1, 64, 17>(sh.Ed2, lg4, l16, true, bias_r, tw, tw2, tb0, tb1);
      float4 aux[4][1] = {};
      conv2_epilogue<4, 1, 1, 1>(d2, rb, 0, lg4, l16, acc, aux, bias_r, tw, tb0, 1.0f, true, rlo, rhi, nullptr, 0, tw2,
                                 tb1);
    }
    if constexpr (PROF) {
      if (it == 0) {
        __syncthreads();
        stamp<PROF>(6);
      }
    }
    ++it;
  }
  if constexpr (PROF) {
    __syncthreads();
    stamp<PROF>(7);
    if (threadIdx.x == 0 && blockIdx.x < 256) g_prof[blockIdx.x * 16 + 8] = (unsigned long long)it;
  }
}

static bool prof_on() {
  static const bool v = [] {
    const char* e = getenv("VQHMM_STRIP_PROF");
    return e && atoi(e) != 0;
  }();
  return v;
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

int launch_strip_fwd(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2, hipStream_t s) {
  if (!strip_fwd_supported(e1, e2, d1, d2)) return VQHMM_EUNSUPPORTED;
  const int64_t nstrip = cdiv(e1.R, ST_OWN);
  const unsigned grid = (unsigned)(nstrip < 256 ? nstrip : 256);
#define VQHMM_SF(NB2, P) strip_fwd_kernel<NB2, P><<<grid, 512, sizeof(StripFwdLds<NB2>), s>>>(e1, e2, d1, d2, nstrip)
  const bool prof = prof_on();
  if (c2_nb(e2.N) == 1) {
    if (prof) VQHMM_SF(1, true); else VQHMM_SF(1, false);
  } else {
    if (prof) VQHMM_SF(2, true); else VQHMM_SF(2, false);
  }
#undef VQHMM_SF
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm

extern "C" int vqhmm_debug_prof(uint64_t* out, int64_t n) {
  if (!out || n < 0 || n > 256 * 16) return VQHMM_EINVAL;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vqhmm::g_prof), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return VQHMM_ELAUNCH;
  return VQHMM_OK;
}
