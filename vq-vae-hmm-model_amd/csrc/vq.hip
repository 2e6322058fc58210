// VQ nearest-neighbour quantization: idx[b,t] = argmin_k ||z[b,:,t] - c[k,:]||^2.
//
// Semantics (no reference code exists): pseudocode.txt:11
// `quantize(z_e, codebook)` and the hard-regime argmax of backtesting.py:154-155.
// Exact contract (oracle/hmm_ref.py, oracle/c/hmm_oracle.c), the expansion form
// ||z||^2 + ||c_k||^2 - 2 z.c_k of SURVEY.md §8d:
//   cn_k = fmaf chain over d of c_kd^2 from +0,
//   s_k  = fmaf chain over d = 0..Dv-1 of z_d * (-2 c_kd) starting from cn_k,
//   idx  = first k with the smallest s_k,  dmin = s_idx + ((q0 + q1) + (q2 + q3))
// where q_r is the fmaf chain of z_d^2 over d = r (mod 4).  A f32 MFMA is
// bit-for-bit a k-ordered fmaf chain, so the matrix cores evaluate s_k exactly.
//
// Main kernel (K <= 32, Dv <= 64 — cfg2 and cfg3):
//  * one v_mfma_f32_32x32x2_f32 per pair of dims: A = the codebook pre-scaled by
//    -2 (32 codes x 2 dims, resident in VGPRs for the whole launch), B = the z
//    tile (2 dims x 32 positions), C starts at cn_k;
//  * every lane loads one dword per dim pair: each wave load is two 128-B
//    segments of the channels-first z; the next tile is prefetched into
//    registers while the MFMAs of the current one run;
//  * the argmin is 15 in-lane compares + one lane^32 exchange (lowest code on
//    ties); the VALU only does the argmin and the ||z||^2 chains.
// Fallback (K > 32 or Dv > 64): VALU kernel over LDS codebook blocks, same chain.
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

namespace vqhmm {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int S>  // MFMA steps of 2 dims each, 2*S >= Dv
__global__ __launch_bounds__(256) void vq_mfma_kernel(const float* __restrict__ z, int64_t B, int Dv, int T,
                                                      const float* __restrict__ cb, int K, int32_t* __restrict__ idx,
                                                      float* __restrict__ dmin, int64_t tiles) {
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int64_t N = B * (int64_t)T;
  const int64_t wave0 = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;

  auto load = [&](int64_t tile, float* zr) {
    int64_t p = tile * 32 + j;
    p = p < N ? p : N - 1;  // clamped address; the result of a clamped lane is not stored
    const int64_t b = p / T;
    const float* base = z + b * (int64_t)Dv * T + (p - b * T);
#pragma unroll
    for (int s = 0; s < S; ++s) zr[s] = base[(int64_t)min(2 * s + h, Dv - 1) * T];  // padded dims: a = 0
  };
  float zc[S];
  if (wave0 < tiles) load(wave0, zc);  // first tile in flight during the codebook prologue

  // A fragments: code j, dim 2s+h, pre-scaled by -2 (exact).  Loads first from
  // clamped addresses (all in flight together), masks after.
  const int jc = min(j, K - 1);
  float a[S];
#pragma unroll
  for (int s = 0; s < S; ++s) a[s] = cb[(int64_t)jc * Dv + min(2 * s + h, Dv - 1)];
#pragma unroll
  for (int s = 0; s < S; ++s) a[s] = (j < K && 2 * s + h < Dv) ? -2.0f * a[s] : 0.0f;
  // cn_j = chain over d ascending: even dims live in lane h=0, odd in h=1
  float cn = 0.0f;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float o = __shfl_xor(a[s], 32);
    const float ce = -0.5f * (h ? o : a[s]), co = -0.5f * (h ? a[s] : o);
    if (2 * s < Dv) cn = __builtin_fmaf(ce, ce, cn);
    if (2 * s + 1 < Dv) cn = __builtin_fmaf(co, co, cn);
  }
  if (j >= K) cn = __builtin_inff();
  // C/D rows of this lane: code i(v) = (v & 3) + 8 (v >> 2) + 4 h, ascending in v
  float init[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) init[v] = __shfl(cn, (v & 3) + 8 * (v >> 2) + 4 * h);

  for (int64_t tile = wave0; tile < tiles; tile += nwaves) {
    float zn[S];
    const bool more = tile + nwaves < tiles;
    if (more) load(tile + nwaves, zn);
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = init[v];
#pragma unroll
    for (int s = 0; s < S; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], zc[s], acc, 0, 0, 0);
    // ||z||^2 partial chains: lane h holds d = 2s+h, i.e. d mod 4 = h (s even) or
    // 2+h (s odd); zn = (q0 + q1) + (q2 + q3)
    float qa = 0.0f, qb = 0.0f;  // d mod 4 = h, 2 + h
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float zv = (2 * s + h < Dv) ? zc[s] : 0.0f;
      if (2 * s < Dv) {
        if (s & 1) qb = __builtin_fmaf(zv, zv, qb);
        else qa = __builtin_fmaf(zv, zv, qa);
      }
    }
    const float pqa = __shfl_xor(qa, 32), pqb = __shfl_xor(qb, 32);
    const float zp = (qa + pqa) + (qb + pqb);
    float best = __builtin_inff();
    int arg = 4 * h;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      if (acc[v] < best) { best = acc[v]; arg = (v & 3) + 8 * (v >> 2) + 4 * h; }
    }
    const float pb = __shfl_xor(best, 32);
    const int pa = __shfl_xor(arg, 32);
    if (pb < best || (pb == best && pa < arg)) { best = pb; arg = pa; }
    const int64_t p = tile * 32 + j;
    if (h == 0 && p < N) {
      idx[p] = arg;
      if (dmin) dmin[p] = best + zp;
    }
    if (more) {
#pragma unroll
      for (int s = 0; s < S; ++s) zc[s] = zn[s];
    }
  }
}

// Row-load variant (T % 4 == 0, Dv % 4 == 0): a 64-position tile per wave, lane
// (g, j) = (lane >> 4, lane & 15) loads float4 z[d = 4 dg + g][t .. t+3] of
// positions 4j .. 4j+3 (each wave load = four 256-B row runs).
// v_mfma_f32_16x16x4_f32 m (m = 0..3) takes component m as B[k = g][col j] =
// z[4 dg + g][position 4j + m]; A = -2 c[16 cb + j][4 dg + g] (from LDS).
// CB x 4 independent accumulators per tile.  Loads are buffer loads: one VGPR
// byte offset per tile + the dim-group offset 16 T dg as an SGPR.  Each wave
// walks a contiguous range of tiles (lines shared by neighbouring tiles stay
// in one XCD's L2).  Two register sets ping-pong: ALL loads of tile n+1 are
// issued before the MFMAs of tile n, so a whole tile of MFMA work covers their
// latency (with one set the compiler sinks the reloads behind the MFMAs that
// read the registers and the wave drains its loads at the top of every tile).
// ||z||^2 (only for dmin) is formed after the MFMAs, so it never pulls a wait
// forward.
// QUANT (quantize, pseudocode.txt:12-18): the epilogue also gathers z_q = c[idx] from an LDS copy of
// the codebook, writes the straight-through value z + (z_q - z) channels-first (float4 stores at the
// z load addresses) and accumulates sum (z - z_q)^2 in the direct-difference form, in fp64, per lane;
// every wave writes one partial (part[global wave]), summed in a fixed order by vq_sse_finalize.
template <int DG, int CB, bool DMIN, int NBUF, bool QUANT = false>  // Dv == 4 DG, K <= 16 CB; DMIN: dmin requested; NBUF register sets
__global__ __launch_bounds__(256, NBUF == 2 ? 2 : 1) void vq_rows_kernel(const float* __restrict__ z, int64_t B, int Dv, int T,
                                                         const float* __restrict__ cb, int K,
                                                         int32_t* __restrict__ idx, float* __restrict__ dmin,
                                                         int64_t tiles, int64_t nwaves, float* __restrict__ zq_st = nullptr,
                                                         double* __restrict__ part = nullptr) {
  constexpr int LDSC = 16 * CB + 4;  // score rows [position][code]
  struct Prologue {
    float cbS[16 * CB][4 * DG + 1];  // codebook, +1 pad: conflict-free per-code rows
  };
  struct Loop {
    float scS[4][64 * LDSC];  // per-wave score transpose
    float qS[4][64 * 4];      // per-wave ||z||^2 partials [position][residue]
  };
  __shared__ union {
    Prologue pro;
    Loop loop;
  } u;
  __shared__ float aS[CB][DG][64];
  __shared__ float cnS[16 * CB];
  __shared__ float cbQ[QUANT ? 16 * CB : 1][QUANT ? 4 * DG : 1];  // QUANT: the codebook, [code][dim]
  __shared__ int argS[QUANT ? 4 : 1][QUANT ? 64 : 1];               // QUANT: the wave's argmins per position
  auto& cbS = u.pro.cbS;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t N = B * (int64_t)T;

  const uint32_t nbytes = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(N * Dv * 4));
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)z, (short)0, (int)nbytes, 0x00020000);
  const int gstep = __builtin_amdgcn_readfirstlane(16 * T);  // bytes between dim groups
  const uint32_t goff = (uint32_t)g * (uint32_t)T * 4u;
  auto tile_off = [&](int64_t tile) -> uint32_t {
    int64_t n = tile * 64 + 4 * j;
    n = n < N ? n : N - 4;  // clamped address; clamped lanes store nothing
    const int64_t b = n / T;
    return (uint32_t)((b * (int64_t)Dv * T + (n - b * T)) * 4) + goff;
  };
  auto load_tile = [&](int64_t tile, f32x4* zr) {
    const uint32_t o = tile_off(tile);
#pragma unroll
    for (int dg = 0; dg < DG; ++dg)
      zr[dg] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rz, (int)o, dg * gstep, 0));
  };

  constexpr int NC = 16 * CB * 4 * DG, NCP = (NC + 255) / 256;
  float cbv[NCP];
#pragma unroll
  for (int k = 0; k < NCP; ++k) cbv[k] = cb[min(tid + 256 * k, K * Dv - 1)];

  const int64_t gw = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(tid >> 6);
  // equal share of the tiles per wave (every resident wave gets floor or ceil of tiles / nwaves)
  const int64_t t0 = gw < nwaves ? tiles * gw / nwaves : tiles;
  const int64_t t1 = gw < nwaves ? tiles * (gw + 1) / nwaves : tiles;
  f32x4 za[DG], zb[DG], zc3[NBUF == 3 ? DG : 1];
  auto clampt = [&](int64_t t) { return t < t1 ? t : (t0 < t1 ? t1 - 1 : 0); };
  load_tile(clampt(t0), za);  // unconditional: in flight during the prologue
  if constexpr (NBUF == 3) load_tile(clampt(t0 + 1), zb);
  // prologue: the codebook crosses HBM once per workgroup (coalesced), then the
  // A fragments and the ||c||^2 chains are built from LDS
#pragma unroll
  for (int k = 0; k < NCP; ++k) {
    const int i = tid + 256 * k;
    if (i < NC) cbS[i / (4 * DG)][i % (4 * DG)] = (i / (4 * DG)) < K ? cbv[k] : 0.0f;
  }
  lds_barrier();
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < CB * DG * 64; i += 256) {
    const int c = i / (DG * 64), dg = (i / 64) % DG, l = i & 63;
    aS[c][dg][l] = -2.0f * cbS[16 * c + (l & 15)][4 * dg + (l >> 4)];
  }
  if constexpr (QUANT)
    for (int i = tid; i < 16 * CB * 4 * DG; i += 256) cbQ[i / (4 * DG)][i % (4 * DG)] = cbS[i / (4 * DG)][i % (4 * DG)];
  if (tid < 16 * CB) {
    float cn = 0.0f;
#pragma unroll
    for (int d = 0; d < 4 * DG; ++d) cn = __builtin_fmaf(cbS[tid][d], cbS[tid][d], cn);
    cnS[tid] = tid < K ? cn : __builtin_inff();
  }

  lds_barrier();
  float init[CB][4];
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int v = 0; v < 4; ++v) init[c][v] = cnS[16 * c + 4 * g + v];
  double sse = 0.0;  // QUANT: sum (z - z_q)^2 of this lane's (position, dim) entries

  // one tile on zc while the loads of tile + NBUF - 1 land in zn
  auto run_tile = [&](int64_t tile, const f32x4* zc, f32x4* zn) {
    load_tile(clampt(tile + NBUF - 1), zn);  // unconditional: keeps the vmcnt counts exact
    __builtin_amdgcn_sched_barrier(0);                 // pin: the loads go out before the MFMAs
    f32x4 acc[CB][4];
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[c][m] = f32x4{init[c][0], init[c][1], init[c][2], init[c][3]};
#pragma unroll
    for (int dg = 0; dg < DG; ++dg) {
      float av[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) av[c] = aS[c][dg][lane];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[c][m] = mfma16x16x4(av[c], zc[dg][m], acc[c][m]);
    }
    // scores through LDS as [position][code] so each lane scans ONE position's
    // codes in ascending order (strict <: lowest code wins ties); position
    // p = 4j + m, code = 16c + 4g + v
    float* sc = u.loop.scS[wave];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int c = 0; c < CB; ++c) *reinterpret_cast<f32x4*>(sc + (4 * j + m) * LDSC + 16 * c + 4 * g) = acc[c][m];
    }
    if constexpr (DMIN) {
      float q[4] = {0.f, 0.f, 0.f, 0.f};  // ||z||^2 chain of residue d = g (mod 4), per position m
#pragma unroll
      for (int dg = 0; dg < DG; ++dg)
#pragma unroll
        for (int m = 0; m < 4; ++m) q[m] = __builtin_fmaf(zc[dg][m], zc[dg][m], q[m]);
#pragma unroll
      for (int m = 0; m < 4; ++m) u.loop.qS[wave][(4 * j + m) * 4 + g] = q[m];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    float best = __builtin_inff();
    int arg = 0;
#pragma unroll
    for (int c4 = 0; c4 < 4 * CB; ++c4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(sc + lane * LDSC + 4 * c4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (v[e] < best) { best = v[e]; arg = 4 * c4 + e; }
    }
    const int64_t n = tile * 64 + lane;
    if (n < N) {
      idx[n] = arg;
      if constexpr (DMIN) {
        const f32x4 qq = *reinterpret_cast<const f32x4*>(&u.loop.qS[wave][lane * 4]);
        dmin[n] = best + ((qq[0] + qq[1]) + (qq[2] + qq[3]));
      }
    }
    if constexpr (QUANT) {
      // lane (g, j) holds z[d = 4 dg + g][positions 4j .. 4j+3]: their codes from the wave's argmins
      argS[wave][lane] = arg;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      int code[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) code[m] = argS[wave][4 * j + m];
      const bool live = tile < t1 && tile * 64 + 4 * j < N;  // T % 4 == 0: a quad is all in or all out
      const uint32_t o = tile_off(tile);
#pragma unroll
      for (int dg = 0; dg < DG; ++dg) {
        f32x4 st;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const float zv = zc[dg][m], qv = cbQ[code[m]][4 * dg + g];
          st[m] = zv + (qv - zv);  // z_e + (z_q - z_e).detach(), :13 (built without contraction)
          const double dd = (double)zv - (double)qv;
          if (live) sse = __builtin_fma(dd, dd, sse);
        }
        if (live) *reinterpret_cast<f32x4*>(reinterpret_cast<char*>(zq_st) + o + (uint32_t)dg * (uint32_t)gstep) = st;
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next tile's writes must not pass this tile's reads
  };
  int64_t tile = t0;
  if constexpr (NBUF == 2) {
    for (; tile + 1 < t1; tile += 2) {  // no branch inside the pair: one pending-load state at the latch
      run_tile(tile, za, zb);
      run_tile(tile + 1, zb, za);
    }
    if (tile < t1) run_tile(tile, za, zb);
  } else {
    for (; tile + 2 < t1; tile += 3) {
      run_tile(tile, za, zc3);
      run_tile(tile + 1, zb, za);
      run_tile(tile + 2, zc3, zb);
    }
    if (tile < t1) run_tile(tile, za, zc3);
    if (tile + 1 < t1) run_tile(tile + 1, zb, za);
  }
  if constexpr (QUANT) {
    sse = wave_sum_dpp(sse);
    if (lane == 0 && gw < nwaves) part[gw] = sse;
  }
}

// ---------------------------------------------------------------- VALU fallback
constexpr int VQ_DCH = 16;

template <int KB>
__global__ __launch_bounds__(256) void vq_argmin_kernel(const float* __restrict__ z, int64_t B, int Dv, int T,
                                                        const float* __restrict__ cb, int K, int ldc,
                                                        int32_t* __restrict__ idx, float* __restrict__ dmin) {
  extern __shared__ float4 cbs4[];
  float* cbs = reinterpret_cast<float*>(cbs4);  // [KB][ldc] = -2 c, ldc = Dv rounded up to 16
  __shared__ float cns[KB];
  const int64_t N = B * (int64_t)T;
  const int lane = threadIdx.x & 63;
  const int64_t n0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 128;
  const int64_t na = n0 + lane, nb = n0 + 64 + lane;
  const bool va = na < N, vb = nb < N;
  const int64_t ba = va ? na / T : 0, bb = vb ? nb / T : 0;
  const float* za = z + ba * (int64_t)Dv * T + (va ? na - ba * T : 0);
  const float* zb = z + bb * (int64_t)Dv * T + (vb ? nb - bb * T : 0);

  float best_a = __builtin_inff(), best_b = __builtin_inff();
  int arg_a = 0, arg_b = 0;
  float qa[4] = {0.f, 0.f, 0.f, 0.f}, qb[4] = {0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < K; kb += KB) {
    const int kn = min(KB, K - kb);
    __syncthreads();
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
    for (int i = threadIdx.x; i < KB * ldc; i += 256) {
      const int k = i / ldc, d = i - k * ldc;
      cbs[i] = (k < kn && d < Dv) ? -2.0f * cb[(int64_t)(kb + k) * Dv + d] : 0.0f;
    }
    if (threadIdx.x < KB) {
      float c2 = 0.f;
      if ((int)threadIdx.x < kn)
        for (int d = 0; d < Dv; ++d) {
          const float c = cb[(int64_t)(kb + threadIdx.x) * Dv + d];
          c2 = __builtin_fmaf(c, c, c2);
        }
      cns[threadIdx.x] = c2;
    }
    __syncthreads();
    float acc_a[KB], acc_b[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) acc_a[k] = acc_b[k] = cns[k];
    for (int dc = 0; dc < Dv; dc += VQ_DCH) {
      const int dn = min(VQ_DCH, Dv - dc);
      for (int d = 0; d < dn; ++d) {
        const float zva = va ? za[(int64_t)(dc + d) * T] : 0.0f;
        const float zvb = vb ? zb[(int64_t)(dc + d) * T] : 0.0f;
        if (kb == 0) {
          const int r = (dc + d) & 3;
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            if (rr == r) { qa[rr] = __builtin_fmaf(zva, zva, qa[rr]); qb[rr] = __builtin_fmaf(zvb, zvb, qb[rr]); }
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const float c = cbs[k * ldc + dc + d];
          acc_a[k] = __builtin_fmaf(zva, c, acc_a[k]);
          acc_b[k] = __builtin_fmaf(zvb, c, acc_b[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (k < kn) {
        if (acc_a[k] < best_a) { best_a = acc_a[k]; arg_a = kb + k; }
        if (acc_b[k] < best_b) { best_b = acc_b[k]; arg_b = kb + k; }
      }
    }
  }
  if (va) { idx[na] = arg_a; if (dmin) dmin[na] = best_a + ((qa[0] + qa[1]) + (qa[2] + qa[3])); }
  if (vb) { idx[nb] = arg_b; if (dmin) dmin[nb] = best_b + ((qb[0] + qb[1]) + (qb[2] + qb[3])); }
}

// ------------------------------------------------- quantize epilogue for the other argmin kernels
// One thread per position (consecutive t: coalesced CF reads / writes): z_q = c[idx], the
// straight-through value z + (z_q - z), and sum (z - z_q)^2 (fp64, direct difference); the block's
// sum goes to part[blockIdx.x] (fixed-order tree).
__global__ __launch_bounds__(256) void vq_quantize_gather_kernel(const float* __restrict__ z, int64_t B, int Dv, int T,
                                                                 const float* __restrict__ cb,
                                                                 const int32_t* __restrict__ idx,
                                                                 float* __restrict__ zq_st, double* __restrict__ part) {
  __shared__ double red[256];
  const int64_t N = B * (int64_t)T;
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double sse = 0.0;
  if (n < N) {
    const int64_t b = n / T, t = n - b * T;
    const int k = idx[n];
    const float* zr = z + b * (int64_t)Dv * T + t;
    float* zo = zq_st + b * (int64_t)Dv * T + t;
    for (int d = 0; d < Dv; ++d) {
      const float zv = zr[(int64_t)d * T], qv = cb[(int64_t)k * Dv + d];
      zo[(int64_t)d * T] = zv + (qv - zv);
      const double dd = (double)zv - (double)qv;
      sse = __builtin_fma(dd, dd, sse);
    }
  }
  red[threadIdx.x] = sse;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// *sse = sum of part[0, np) in a fixed order (one workgroup)
__global__ __launch_bounds__(256) void vq_sse_finalize_kernel(const double* __restrict__ part, int64_t np,
                                                              double* __restrict__ sse) {
  __shared__ double red[256];
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < np; i += 256) v += part[i];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) *sse = red[0];
}

static int env_int(const char* e, int dflt, int lo, int hi) {
  const int v = e ? atoi(e) : dflt;
  return v >= lo && v <= hi ? v : dflt;
}

static int64_t persistent_waves(int64_t tiles, int dflt = 8) {
  static const int wpc = env_int(VQHMM_PROF_ENV("VQHMM_VQ_WPC"), 0, 1, 32);  // tuning knob: resident waves per CU
  return std::min<int64_t>(tiles, 256 * (int64_t)(wpc ? wpc : dflt));
}

template <int S>
static void launch_mfma(const float* z, int64_t B, int Dv, int T, const float* cb, int K, int32_t* idx, float* dmin,
                        hipStream_t s) {
  const int64_t tiles = cdiv(B * (int64_t)T, 32);
  vq_mfma_kernel<S><<<(unsigned)cdiv(persistent_waves(tiles), 4), 256, 0, s>>>(z, B, Dv, T, cb, K, idx, dmin, tiles);
}

static int64_t rows_waves(int64_t N) {  // one wave per SIMD measured best (cfg3)
  return cdiv(persistent_waves(cdiv(N, 64), 4), 4) * 4;
}

template <int DG, int CB>
static void launch_rows(const float* z, int64_t B, int Dv, int T, const float* cb, int K, int32_t* idx, float* dmin,
                        hipStream_t s, float* zq_st = nullptr, double* part = nullptr) {
  static const int nbuf = env_int(VQHMM_PROF_ENV("VQHMM_VQ_NBUF"), 2, 2, 3);  // tuning knob: register sets in flight
  const int64_t tiles = cdiv(B * (int64_t)T, 64);
  const int64_t waves = rows_waves(B * (int64_t)T);
  const unsigned grid = (unsigned)(waves / 4);
  if (zq_st) {
    vq_rows_kernel<DG, CB, false, 2, true><<<grid, 256, 0, s>>>(z, B, Dv, T, cb, K, idx, nullptr, tiles, waves, zq_st,
                                                                part);
    return;
  }
  if (nbuf == 3) {
    if (dmin) vq_rows_kernel<DG, CB, true, 3><<<grid, 256, 0, s>>>(z, B, Dv, T, cb, K, idx, dmin, tiles, waves);
    else vq_rows_kernel<DG, CB, false, 3><<<grid, 256, 0, s>>>(z, B, Dv, T, cb, K, idx, dmin, tiles, waves);
  } else {
    if (dmin) vq_rows_kernel<DG, CB, true, 2><<<grid, 256, 0, s>>>(z, B, Dv, T, cb, K, idx, dmin, tiles, waves);
    else vq_rows_kernel<DG, CB, false, 2><<<grid, 256, 0, s>>>(z, B, Dv, T, cb, K, idx, dmin, tiles, waves);
  }
}

// Dv % 4 == 0 only (whole dim groups)
template <int CB>
static bool dispatch_rows(const float* z, int64_t B, int Dv, int T, const float* cb, int K, int32_t* idx,
                          float* dmin, hipStream_t s, float* zq_st = nullptr, double* part = nullptr) {
  switch (Dv) {
    case 4: launch_rows<1, CB>(z, B, Dv, T, cb, K, idx, dmin, s, zq_st, part); return true;
    case 8: launch_rows<2, CB>(z, B, Dv, T, cb, K, idx, dmin, s, zq_st, part); return true;
    case 16: launch_rows<4, CB>(z, B, Dv, T, cb, K, idx, dmin, s, zq_st, part); return true;
    case 32: launch_rows<8, CB>(z, B, Dv, T, cb, K, idx, dmin, s, zq_st, part); return true;
    case 64: launch_rows<16, CB>(z, B, Dv, T, cb, K, idx, dmin, s, zq_st, part); return true;
    default: return false;
  }
}

static bool rows_path(const float* z, int64_t B, int64_t Dv, int64_t T, int64_t K) {
  static const int impl = env_int(VQHMM_PROF_ENV("VQHMM_VQ_IMPL"), 0, 0, 2);  // 0 auto, 1 tile-32, 2 rows
  const int64_t N = B * T;
  const bool rows_ok = T % 4 == 0 && (reinterpret_cast<uintptr_t>(z) & 15) == 0 && N * Dv < (int64_t(1) << 30);
  return K <= 32 && rows_ok && impl != 1 && (Dv == 4 || Dv == 8 || Dv == 16 || Dv == 32 || Dv == 64);
}

size_t vq_quantize_ws_bytes(int64_t B, int64_t Dv, int64_t T, int64_t K) {
  (void)Dv; (void)K;
  const int64_t N = B * T;
  const int64_t np = std::max<int64_t>(rows_waves(N), cdiv(N, 256));
  return (size_t)std::max<int64_t>(np, 1) * sizeof(double);
}

int launch_vq_quantize(const float* z, int64_t B, int64_t Dv, int64_t T, const float* cb, int64_t K, int32_t* idx,
                       float* zq_st, double* sse, void* ws, size_t ws_bytes, hipStream_t s) {
  const int64_t N = B * T;
  if (K <= 0 || Dv <= 0 || Dv > 2048 || T <= 0 || T > INT32_MAX) return VQHMM_EINVAL;
  if (ws_bytes < vq_quantize_ws_bytes(B, Dv, T, K)) return VQHMM_EWORKSPACE;
  double* part = reinterpret_cast<double*>(ws);
  int64_t np;
  if (N > 0 && rows_path(z, B, Dv, T, K)) {
    const bool done = K <= 16 ? dispatch_rows<1>(z, B, (int)Dv, (int)T, cb, (int)K, idx, nullptr, s, zq_st, part)
                              : dispatch_rows<2>(z, B, (int)Dv, (int)T, cb, (int)K, idx, nullptr, s, zq_st, part);
    if (!done) return VQHMM_EUNSUPPORTED;
    np = rows_waves(N);
  } else {
    if (int rc = launch_vq_argmin(z, B, Dv, T, cb, K, idx, nullptr, s)) return rc;
    np = cdiv(N, 256);
    if (np > 0)
      vq_quantize_gather_kernel<<<(unsigned)np, 256, 0, s>>>(z, B, (int)Dv, (int)T, cb, idx, zq_st, part);
  }
  VQHMM_LAUNCH_CHECK();
  vq_sse_finalize_kernel<<<1, 256, 0, s>>>(part, np, sse);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_vq_argmin(const float* z, int64_t B, int64_t Dv, int64_t T, const float* cb, int64_t K,
                     int32_t* idx, float* dmin, hipStream_t s) {
  const int64_t N = B * T;
  if (N == 0) return VQHMM_OK;
  if (K <= 0 || Dv <= 0 || Dv > 2048 || T <= 0 || T > INT32_MAX) return VQHMM_EINVAL;
  static const int impl = env_int(VQHMM_PROF_ENV("VQHMM_VQ_IMPL"), 0, 0, 2);  // 0 auto, 1 tile-32, 2 rows
  const bool rows_ok = T % 4 == 0 && (reinterpret_cast<uintptr_t>(z) & 15) == 0 && N * Dv < (int64_t(1) << 30);
  if (K <= 32 && Dv <= 64 && rows_ok && impl != 1) {
    const bool done = K <= 16 ? dispatch_rows<1>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s)
                              : dispatch_rows<2>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s);
    if (done) {
      VQHMM_LAUNCH_CHECK();
      return VQHMM_OK;
    }
  }
  if (K <= 32 && Dv <= 64) {
    const int S = (int)cdiv(Dv, 2);
    if (S <= 2) launch_mfma<2>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s);
    else if (S <= 4) launch_mfma<4>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s);
    else if (S <= 8) launch_mfma<8>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s);
    else if (S <= 16) launch_mfma<16>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s);
    else launch_mfma<32>(z, B, (int)Dv, (int)T, cb, (int)K, idx, dmin, s);
    VQHMM_LAUNCH_CHECK();
    return VQHMM_OK;
  }
  const int ldc = (int)cdiv(Dv, VQ_DCH) * VQ_DCH;
  const dim3 grid((unsigned)cdiv(N, 512));
  int kb = K <= 4 ? 4 : K <= 8 ? 8 : K <= 16 ? 16 : 32;
  while (kb > 4 && (size_t)kb * ldc * 4 > 64 * 1024) kb >>= 1;
  const size_t lds = (size_t)kb * ldc * sizeof(float);
  if (lds > 64 * 1024) return VQHMM_EUNSUPPORTED;
  switch (kb) {
    case 4: vq_argmin_kernel<4><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
    case 8: vq_argmin_kernel<8><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
    case 16: vq_argmin_kernel<16><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
    default: vq_argmin_kernel<32><<<grid, 256, lds, s>>>(z, B, (int)Dv, (int)T, cb, (int)K, ldc, idx, dmin); break;
  }
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm
