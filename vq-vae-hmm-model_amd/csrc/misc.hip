// Small kernels of the training step:
//   grad_tail        deterministic split-K reduction of the per-workgroup gradient slabs into
//                    the flat gradient (fixed chunk order, no atomics) + the log_prior gradient
//   compose_adam     (single process) the composed decoder conv1's dW / dE and every element's
//                    Adam update in the step's last launch
//   finalize_loss    loss = recon + beta*(prior - entropy)  (VQ_VAE_HMM_fixed.py:137)
//   compose_fwd/bwd  decoder embedding folded into decoder.conv1:
//                    conv1(q^T E) == conv1'(q) with W'[o,k,tap] = sum_h W[o,h,tap] E[k,h];
//                    (compose_bwd: the generic path's dW / dE when the tail cannot take them)
//   prologue         x, u -> PCL + compose_fwd in one launch (the step's first stage)
//   logits_bwd       softmax backward of q = softmax(logits) (:114) + entropy's direct term
//   adam             torch.optim.Adam update (defaults of train_model, :146)
#include <algorithm>

#include "kernels.h"

namespace vqhmm {

// ------------------------------------------------------------ backward tail
// torch.optim.Adam's update of element i (adam_kernel below has the derivation and the device
// step counter; tn = this step's count).  Split so a caller can load the element's state early
// (adam_load) and apply it once the gradient is known (adam_apply).  misc.hip is built with
// -ffp-contract=off, so every launch that applies it rounds identically.
struct AdamElem {
  float step_size, bc2s, m, v, p;
};
__device__ __forceinline__ AdamElem adam_load(const AdamArgs& a, int64_t i, int64_t tn) {
  const double t = (double)tn;
  AdamElem e;
  e.step_size = (float)(a.lr / (1.0 - pow(a.b1, t)));
  e.bc2s = (float)sqrt(1.0 - pow(a.b2, t));
  e.m = a.m[i];
  e.v = a.v[i];
  e.p = a.p[i];
  return e;
}
struct AdamOut {
  float m, v, p;
};
__device__ __forceinline__ AdamOut adam_elem(const AdamArgs& a, float g, const AdamElem& e) {
  const float gi = g * a.gmul;
  const float mi = e.m + (float)(1.0 - a.b1) * (gi - e.m);
  const float vi = e.v * (float)a.b2 + (float)(1.0 - a.b2) * gi * gi;
  const float denom = sqrtf(vi) / e.bc2s + (float)a.eps;
  return AdamOut{mi, vi, e.p + (-e.step_size) * (mi / denom)};
}
__device__ __forceinline__ void adam_apply(const AdamArgs& a, int64_t i, float g, const AdamElem& e) {
  const AdamOut o = adam_elem(a, g, e);
  a.m[i] = o.m;
  a.v[i] = o.v;
  a.p[i] = o.p;
}
// The step counter advances inside the update's own launch: every workgroup read
// t = (*step & 0xffffffff) + 1 at its start, then takes a ticket in the upper 32 bits here; the
// last one to do so (all reads are behind it) stores t with a zero ticket.  No fence: the ticket
// orders only the reads of *step, not this workgroup's parameter writes.
__device__ __forceinline__ void adam_ticket(int64_t* step, int64_t tn) {
  __syncthreads();
  if (threadIdx.x == 0) {
    auto* st = reinterpret_cast<unsigned long long*>(step);
    const unsigned long long old = atomicAdd(st, 1ull << 32);
    if ((old >> 32) == gridDim.x - 1) atomicExch(st, (unsigned long long)tn);
  }
}

// Columns [v0, v0 + nv) of a [nch][ld] slab summed over its chunks into red[0, nv) (LDS), by the
// whole workgroup: value v is split over P = 256 / nv chunk phases (16 interleaved partials each),
// combined in a fixed order.  Ends with a barrier.
__device__ void block_reduce_cols(const float* slab, int64_t nch, int64_t ld, int64_t v0, int nv, float* red,
                                  float* scratch) {
  const int tid = threadIdx.x;
  for (int base = 0; base < nv; base += 256) {
    const int n = min(256, nv - base);
    const int P = 256 / n;
    const int v = tid % n, ph = tid / n;
    if (ph < P) {  // 16 loads in flight per round: the chunk loop is latency-bound
      float acc[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      const float* col = slab + v0 + base + v;
      int64_t c = ph;
      for (; c + 15 * P < nch; c += 16 * P)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] += col[(c + j * P) * ld];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (c + j * P < nch) acc[j] += col[(c + j * P) * ld];
#pragma unroll
      for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int j = 0; j < w; ++j) acc[j] += acc[j + w];
      scratch[ph * n + v] = acc[0];
    }
    __syncthreads();
    if (tid < n) {
      float r = 0.f;
      for (int h = 0; h < P; ++h) r += scratch[h * n + tid];
      red[base + tid] = r;
    }
    __syncthreads();
  }
}

// Columns [64 (blockIdx.x - blk_start[si]), +64) of segment si summed over its chunks (fixed order)
// and written to sg.out; returns the segment index (the caller's block is one of its blocks).
// Threads < 64 hold their column's value in *val (valid when *col < len).
// Composed segment (SlabSeg::cmpE): the block's 64 columns of dW lie in o rows o_lo .. o_hi; it reduces
// those rows' dWc columns (3K each, contiguous in the slab) over the chunks itself, then forms
// dW[o][h][tap] = sum_k dWc[o][k][tap] E[k][h] (fmaf chain over k, as compose_adam_block).
__device__ void tail_composed_block(const SlabSeg& sg, int64_t col0, float* red, float* scratch, float* val,
                                    int64_t* colp) {
  const int H = sg.cmpH, K = sg.cmpK, L3 = 3 * K;
  const int64_t o_lo = col0 / (3 * H), o_hi = min(col0 + 63, sg.len - 1) / (3 * H);
  block_reduce_cols(sg.slab, sg.nchunks, (int64_t)H * L3, o_lo * L3, (int)((o_hi - o_lo + 1) * L3), red, scratch);
  const int64_t col = col0 + threadIdx.x;
  if (threadIdx.x < 64 && col < sg.len) {
    const int o = (int)(col / (3 * H)), rem = (int)(col - (int64_t)o * 3 * H), h = rem / 3, tap = rem - 3 * h;
    const float* dwc = red + (o - o_lo) * L3;
    float v = 0.f;
    for (int k = 0; k < K; ++k) v = fmaf(dwc[k * 3 + tap], sg.cmpE[(int64_t)k * H + h], v);
    if (sg.scale) v *= *sg.scale;
    sg.out[col] = v;
    *val = v;
  }
  *colp = col;
}

__device__ int tail_segment_block(const TailArgs& ta, float (&part)[16][64], float* red, float* scratch, float* val,
                                  int64_t* colp) {
  int si = 0;
  while (si + 1 < ta.nseg && (int64_t)blockIdx.x >= ta.blk_start[si + 1]) ++si;
  const SlabSeg& sg = ta.s[si];
  const int64_t col0 = ((int64_t)blockIdx.x - ta.blk_start[si]) * 64;
  if (sg.cmpE) {
    tail_composed_block(sg, col0, red, scratch, val, colp);
    return si;
  }
  const bool vec = (sg.len % 4 == 0) && ((reinterpret_cast<uintptr_t>(sg.slab) & 15) == 0);
  int nph;
  if (vec) {
    nph = 16;
    const int ph = threadIdx.x >> 4, cg = (threadIdx.x & 15) * 4;
    const int64_t c4 = col0 + cg;
    float4 p8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) p8[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < sg.len) {  // len % 4 == 0: the whole float4 is in range
      const float4* sl = reinterpret_cast<const float4*>(sg.slab + c4);
      const int64_t ld = sg.len / 4;
      int64_t c = ph;
      for (; c + 112 < sg.nchunks; c += 128) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float4 v = sl[(c + 16 * k) * ld];
          p8[k].x += v.x; p8[k].y += v.y; p8[k].z += v.z; p8[k].w += v.w;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // < 8 rows left per phase
        if (c + 16 * k < sg.nchunks) {
          const float4 v = sl[(c + 16 * k) * ld];
          p8[k].x += v.x; p8[k].y += v.y; p8[k].z += v.z; p8[k].w += v.w;
        }
      }
    }
    float acc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      auto g = [&](int k) { return e == 0 ? p8[k].x : e == 1 ? p8[k].y : e == 2 ? p8[k].z : p8[k].w; };
      acc[e] = ((g(0) + g(1)) + (g(2) + g(3))) + ((g(4) + g(5)) + (g(6) + g(7)));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) part[ph][cg + e] = acc[e];
  } else {
    nph = 4;
    const int64_t cs = col0 + (threadIdx.x & 63);
    const int ph = threadIdx.x >> 6;
    float p8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cs < sg.len) {
      int64_t c = ph;
      for (; c + 28 < sg.nchunks; c += 32) {
#pragma unroll
        for (int k = 0; k < 8; ++k) p8[k] += sg.slab[(c + 4 * k) * sg.len + cs];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)  // < 8 rows left per phase
        if (c + 4 * k < sg.nchunks) p8[k] += sg.slab[(c + 4 * k) * sg.len + cs];
    }
    part[ph][threadIdx.x & 63] = ((p8[0] + p8[1]) + (p8[2] + p8[3])) + ((p8[4] + p8[5]) + (p8[6] + p8[7]));
  }
  __syncthreads();
  const int64_t col = col0 + threadIdx.x;
  if (threadIdx.x < 64 && col < sg.len) {
    float v = 0.f;
    for (int h = 0; h < nph; h += 4)
      v += ((part[h][threadIdx.x] + part[h + 1][threadIdx.x]) + part[h + 2][threadIdx.x]) + part[h + 3][threadIdx.x];
    if (sg.scale) v *= *sg.scale;
    sg.out[seg_out_index(sg, col)] = v;
    *val = v;
  }
  *colp = col;
  return si;
}

// log_prior gradient (VQ_VAE_HMM_fixed.py:71,:123,:131) from the q0 slab, and (ADAM) its Adam update:
// thread k < K owns element k; its log_prior value and Adam operands are loaded before the slab reduction,
// thread 0 forms the max / sum terms from LDS in the fixed order (k ascending).
template <bool ADAM>
__device__ void tail_logprior_block(const TailArgs& ta, float* red, float* scratch, const AdamArgs& ad, int64_t tn,
                                    const float* g) {
  const LogPriorGradArgs& lp = ta.lp;
  const int K = lp.K, tid = threadIdx.x;
  __shared__ float lsum[3];
  const float lpk = tid < K ? lp.log_prior[tid] : 0.f;
  AdamElem e{};
  if (ADAM && tid < K) e = adam_load(ad, (lp.out - g) + tid, tn);
  block_reduce_cols(ta.q0slab, ta.q0chunks, K, 0, K, red, scratch);  // ends with a barrier
  if (tid < K) scratch[tid] = lpk;
  __syncthreads();
  const float c = -lp.beta / loss_norm_batch(lp.norm, lp.B);
  if (tid == 0) {
    float m = -__builtin_inff();
    for (int k = 0; k < K; ++k) m = fmaxf(m, scratch[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += __expf(scratch[k] - m);
    float tot = 0.f;
    for (int k = 0; k < K; ++k) tot += c * red[k];
    lsum[0] = m;
    lsum[1] = se;
    lsum[2] = tot;
  }
  __syncthreads();
  if (tid < K) {
    const float sc = lp.scale ? *lp.scale : 1.f;
    const float v = sc * (c * red[tid] - __expf(lpk - lsum[0]) / lsum[1] * lsum[2]);
    lp.out[tid] = v;
    if constexpr (ADAM) adam_apply(ad, (lp.out - g) + tid, v, e);
  }
}

// grad_tail (the tail without Adam) is tail_kernel<false>: one workgroup = 64 consecutive columns of one
// segment x all its chunks (where a segment's rows are float4-aligned, 16 lanes x float4 cover the 64
// columns and 16 chunk phases keep 16 x 8 wide loads in flight per column group; otherwise 64 lanes x 4
// phases of scalar loads), or (q0slab set) the log_prior gradient, or the loss finalize.  Phases combine in
// a fixed order.

// The non-grouped path's composed decoder conv1 from the reduced dWc: element block cb < cdiv(H*H*3, 256)
// of dW (256 elements), else row k = cb - that of dE (4 thread groups splitting o, combined in a fixed
// order); gradient into g, then (ADAM) Adam.  pre: this thread's Adam element of a dW block, already
// loaded (or null)
template <bool ADAM>
__device__ void compose_adam_block(const ComposeAdamArgs& a, int64_t cb, int64_t tn, float (&part)[4][256],
                                   const AdamElem* pre = nullptr) {
  const AdamArgs& ad = a.adam;
  const int H = a.H, K = a.K;
  const int64_t nw = cdiv((int64_t)H * H * 3, 256);
  if (cb < nw) {
    const int64_t j = cb * 256 + threadIdx.x;
    if (j < (int64_t)H * H * 3) {
      const int64_t i = a.off_w + j;
      AdamElem e{};
      if constexpr (ADAM) e = pre ? *pre : adam_load(ad, i, tn);
      const int o = (int)(j / (3 * H)), rem = (int)(j - (int64_t)o * 3 * H), h = rem / 3, tap = rem - 3 * h;
      float sacc = 0.f;
#pragma unroll 4
      for (int k = 0; k < K; ++k) sacc = fmaf(a.dWc[((int64_t)o * K + k) * 3 + tap], a.Ecopy[(int64_t)k * H + h], sacc);
      a.g[i] = sacc;
      if constexpr (ADAM) adam_apply(ad, i, sacc, e);
    }
    return;
  }
  // one block per (k, 64-wide h chunk): one block per k walked its H / 64 chunks one after another, each a
  // chain of dependent load batches (cfg3: 32 blocks x 4 chunks, most of the 149 us launch)
  const int nh = (int)cdiv(H, 64);
  const int k = (int)((cb - nw) / nh), h0 = (int)((cb - nw) % nh) * 64;
  const int grp = threadIdx.x >> 6;
  {
    const int h = h0 + (threadIdx.x & 63);
    float sacc = 0.f;
    if (h < H)
#pragma unroll 8  // loads of 8 o-steps in flight; the fma chain order is unchanged
      for (int o = grp; o < H; o += 4)
#pragma unroll
        for (int tap = 0; tap < 3; ++tap)
          sacc = fmaf(a.dWc[((int64_t)o * K + k) * 3 + tap], a.Wcopy[((int64_t)o * H + h) * 3 + tap], sacc);
    part[grp][threadIdx.x & 63] = sacc;
    __syncthreads();
    if (threadIdx.x < 64 && h < H) {
      const int64_t i = a.off_e + (int64_t)k * H + h;
      const float gv = ((part[0][threadIdx.x] + part[1][threadIdx.x]) + part[2][threadIdx.x]) + part[3][threadIdx.x];
      a.g[i] = gv;
      if constexpr (ADAM) adam_apply(ad, i, gv, adam_load(ad, i, tn));
    }
    __syncthreads();
  }
}

// Blocks [0, nb): 256 consecutive elements each: Adam on the reduced gradient, except the composed
// decoder conv1 weight / embedding (compose_adam_block), which follow.
__global__ __launch_bounds__(256) void compose_adam_kernel(ComposeAdamArgs a) {
  __shared__ float part[4][256];
  const AdamArgs& ad = a.adam;
  const int64_t tn = (*ad.step & 0xffffffffll) + 1;
  const int64_t nb = cdiv(a.n, 256);
  if ((int64_t)blockIdx.x < nb) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool composed = (i >= a.off_w && i < a.off_w + (int64_t)a.H * a.H * 3) ||
                          (i >= a.off_e && i < a.off_e + (int64_t)a.K * a.H);
    if (i < a.n && !composed) adam_apply(ad, i, a.g[i], adam_load(ad, i, tn));
  } else {
    compose_adam_block<true>(a, (int64_t)blockIdx.x - nb, tn, part);
  }
  adam_ticket(ad.step, tn);
}

// The whole backward tail in ONE launch: grad_tail's blocks, each (ADAM) then applying Adam to the columns
// it has just reduced (their Adam operands are loaded before the reduction).  Block order: [segment
// blocks][log_prior][loss finalize].  Every block works alone: the composed decoder conv1's dW blocks reduce
// their own dWc rows (tail_composed_block) and its dE arrives as a per-chunk slab from the weight-gradient
// launch (WgradArgs::cmp_slab), so no block waits for another and nothing depends on dispatch order.
// ADAM: the step counter was already advanced by an earlier launch of the same backward (the grouped
// weight-gradient launch, WgradGroup::step_inc), so every block reads this step's count as it is: no
// completion ticket (560 same-address atomics cost ~5 us at B = 128).
template <bool ADAM>
__global__ __launch_bounds__(256) void tail_kernel(TailArgs ta, AdamArgs ad, const float* g) {
  __shared__ float part[16][64];
  __shared__ float red[256];
  __shared__ float scratch[256];
  // the step count as a VECTOR load (opaque zero index): a scalar load's cache miss would hold the lgkmcnt(0)
  // before every kernel-argument pointer use (scalar loads return out of order), i.e. every block's first loads
  int z0 = 0;
  asm volatile("" : "+v"(z0));
  const int64_t tn = ADAM ? (ad.step[z0] & 0xffffffffll) : 0;
  const int64_t nblk = ta.blk_start[ta.nseg];
  const int64_t b = blockIdx.x;
  const int64_t finb = nblk + (ta.q0slab ? 1 : 0);
  if (b < nblk) {
    AdamElem e{};
    if constexpr (ADAM) {  // this column's Adam operands in flight across the slab reduction
      int sj = 0;
      while (sj + 1 < ta.nseg && b >= ta.blk_start[sj + 1]) ++sj;
      const int64_t c = (b - ta.blk_start[sj]) * 64 + threadIdx.x;
      if (threadIdx.x < 64 && c < ta.s[sj].len) e = adam_load(ad, (ta.s[sj].out - g) + seg_out_index(ta.s[sj], c), tn);
    }
    float v = 0.f;
    int64_t col;
    int si = 0;
    if (ta.dbg & 1) {
      while (si + 1 < ta.nseg && b >= ta.blk_start[si + 1]) ++si;
      col = (b - ta.blk_start[si]) * 64 + threadIdx.x;
    } else {
      si = tail_segment_block(ta, part, red, scratch, &v, &col);
    }
    const SlabSeg& sg = ta.s[si];
    if (ADAM && !(ta.dbg & 8) && threadIdx.x < 64 && col < sg.len) adam_apply(ad, (sg.out - g) + seg_out_index(sg, col), v, e);
  } else if (ta.q0slab && b == nblk) {
    if (ta.dbg & 2) return;
    tail_logprior_block<ADAM>(ta, red, scratch, ad, tn, g);
  } else if (ta.fin_loss && b == finb) {
    if (ta.dbg & 4) return;
    __shared__ double fred[5 * 256];
    finalize_loss_block(ta.fin_part, ta.fin_nblk, nullptr, ta.lp.norm, ta.fin_B, ta.fin_T, ta.fin_D, ta.lp.beta,
                        ta.fin_loss, ta.fin_accum, ta.fin_pieces, fred, ta.fin_cnt);
  }
}

static void prof_empties(const char* name, hipStream_t s);
int launch_tail(TailArgs& ta, const AdamArgs* adam, const float* g, hipStream_t s) {
  prof_empties("VQHMM_TAIL_EMPTY", s);
  if (ta.nseg > MAX_SEGS || (ta.q0slab && ta.lp.K > 256)) return VQHMM_EINVAL;
  for (int i = 0; i < ta.nseg; ++i)
    if (ta.s[i].cmpE && composed_block_cols(ta.s[i].cmpH, ta.s[i].cmpK) > 256) return VQHMM_EINVAL;
  {
    static const char* dbg = VQHMM_PROF_ENV("VQHMM_TAIL_DBG");
    ta.dbg = dbg ? atoi(dbg) : 0;
  }
  ta.blk_start[0] = 0;
  for (int i = 0; i < ta.nseg; ++i) ta.blk_start[i + 1] = ta.blk_start[i] + cdiv(ta.s[i].len, 64);
  const int64_t nb = ta.blk_start[ta.nseg] + (ta.q0slab ? 1 : 0) + (ta.fin_loss ? 1 : 0);
  if (nb == 0) return VQHMM_OK;
  if (adam)
    tail_kernel<true><<<(unsigned)nb, 256, 0, s>>>(ta, *adam, g);
  else
    tail_kernel<false><<<(unsigned)nb, 256, 0, s>>>(ta, AdamArgs{}, g);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_grad_tail(TailArgs& a, hipStream_t s) { return launch_tail(a, nullptr, nullptr, s); }

int launch_compose_adam(const ComposeAdamArgs& a, hipStream_t s) {
  const int64_t nb = cdiv(a.n, 256) + cdiv((int64_t)a.H * a.H * 3, 256) + (int64_t)a.K * cdiv(a.H, 64);
  compose_adam_kernel<<<(unsigned)nb, 256, 0, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ------------------------------------------------------------ loss finalize
// part[nblk][4] = recon_sum, init_sum, trans_sum, ent_sum (ent_sum = sum of -sum_k q log q).
__global__ void finalize_loss_kernel(const double* part, int nblk, const int64_t* lengths, const int64_t* norm,
                                     int64_t B, int T, int D, float beta, float* loss, double* accum, float* pieces) {
  __shared__ double red[5 * 256];
  finalize_loss_block(part, nblk, lengths, norm, B, T, D, beta, loss, accum, pieces, red);
}

int launch_finalize_loss(const double* part, int nblk, const int64_t* lengths, const int64_t* norm, int64_t B, int T,
                         int D, float beta, float* loss, double* accum, float* pieces, hipStream_t s) {
  finalize_loss_kernel<<<1, 256, 0, s>>>(part, nblk, lengths, norm, B, T, D, beta, loss, accum, pieces);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ------------------------------------------------------------ composed decoder conv1
// Wc[o][k][tap] = sum_h W[o][h][tap] * E[k][h];  W (H,H,3), E (K,H), Wc (H,K,3).
// One block per output channel o; W[o] and E staged in LDS.
// img_f / img_d (nullable): the packed conv2_kernel images of Wc for the forward (N = H, Kc = K)
// and the data gradient (N = K, Kc = H) — this block writes their entries of channel o; the
// image jobs (wimg_slice, composed) write the zero padding around them.
__device__ __forceinline__ void compose_fwd_block(const float* W, const float* E, int H, int K, float* Wc, int o,
                                                  float* cs, float* img_f = nullptr, float* img_d = nullptr,
                                                  float* Ecopy = nullptr, float* Wcopy = nullptr) {
  float* wo = cs;          // [H*3]
  float* es = cs + H * 3;  // [K*H]
  for (int i = threadIdx.x; i < H * 3; i += 256) {
    wo[i] = W[(int64_t)o * H * 3 + i];
    if (Wcopy) Wcopy[(int64_t)o * H * 3 + i] = wo[i];
  }
  for (int i = threadIdx.x; i < K * H; i += 256) {
    es[i] = E[i];
    if (Ecopy && o == 0) Ecopy[i] = es[i];
  }
  __syncthreads();
  // output i = (k, tap) per wave (i = wave, wave + 4, ...): lane l sums h = l, l + 64, ... in order, then a
  // fixed-order wave tree (was one thread per output with an H-long dependent chain: the prologue's longest path)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = wave; i < K * 3; i += 4) {
    const int k = i / 3, tap = i % 3;
    float s = 0.f;
    for (int h = lane; h < H; h += 64) s = fmaf(wo[h * 3 + tap], es[k * H + h], s);
    s = wave_sum_dpp(s);
    if (lane == 0) {
      Wc[(int64_t)o * K * 3 + i] = s;
      if (img_f) img_f[((int64_t)tap * 16 * c2_nb(H) + o) * c2_ldx(K) + k] = s;
      if (img_d) img_d[((int64_t)(2 - tap) * 16 * c2_nb(K) + k) * c2_ldx(H) + o] = s;
    }
  }
}
__global__ __launch_bounds__(256) void compose_fwd_kernel(const float* W, const float* E, int H, int K, float* Wc) {
  extern __shared__ float cs[];
  compose_fwd_block(W, E, H, K, Wc, blockIdx.x, cs);
}
// dW[o][h][tap] = sum_k dWc[o][k][tap] E[k][h]       (blocks 0..H-1, one per o)
// dE[k][h] = sum_{o,tap} dWc[o][k][tap] W[o][h][tap]  (blocks H..H+K-1, one per k;
//            4 thread groups split o, combined in fixed order)
__device__ void log_prior_grad_body(const LogPriorGradArgs& a);

// Block H + K (when lp.out is set) computes the log_prior gradient
// (log_prior_grad_body): both are the step's last, tiny reductions, so they share one launch.
__global__ __launch_bounds__(256) void compose_bwd_kernel(const float* dWc, const float* W, const float* E, int H,
                                                          int K, float* dW, float* dE, LogPriorGradArgs lp) {
  extern __shared__ float cs[];
  if ((int)blockIdx.x == H + K) {
    if (threadIdx.x == 0) log_prior_grad_body(lp);
    return;
  }
  if ((int)blockIdx.x < H) {
    const int o = blockIdx.x;
    float* dwo = cs;           // [K*3]
    float* es = cs + K * 3;    // [K*H]
    for (int i = threadIdx.x; i < K * 3; i += 256) dwo[i] = dWc[(int64_t)o * K * 3 + i];
    for (int i = threadIdx.x; i < K * H; i += 256) es[i] = E[i];
    __syncthreads();
    for (int i = threadIdx.x; i < H * 3; i += 256) {
      const int h = i / 3, tap = i % 3;
      float s = 0.f;
      for (int k = 0; k < K; ++k) s = fmaf(dwo[k * 3 + tap], es[k * H + h], s);
      dW[(int64_t)o * H * 3 + i] = s;
    }
  } else {
    const int k = blockIdx.x - H;
    float* part = cs;  // [4][H]
    const int g = threadIdx.x >> 6;
    for (int h = threadIdx.x & 63; h < H; h += 64) {
      float s = 0.f;
#pragma unroll 8
      for (int o = g; o < H; o += 4)
#pragma unroll
        for (int tap = 0; tap < 3; ++tap)
          s = fmaf(dWc[((int64_t)o * K + k) * 3 + tap], W[((int64_t)o * H + h) * 3 + tap], s);
      part[g * H + h] = s;
    }
    __syncthreads();
    for (int h = threadIdx.x; h < H; h += 256)
      dE[(int64_t)k * H + h] = ((part[h] + part[H + h]) + part[2 * H + h]) + part[3 * H + h];
  }
}

int launch_compose_fwd(const float* W, const float* E, int H, int K, float* Wc, hipStream_t s) {
  const size_t lds = (size_t)(H * 3 + K * H) * 4;
  compose_fwd_kernel<<<(unsigned)H, 256, lds, s>>>(W, E, H, K, Wc);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}
int launch_compose_bwd(const float* dWc, const float* W, const float* E, int H, int K, float* dW, float* dE,
                       const LogPriorGradArgs& lp, hipStream_t s) {
  size_t lds = (size_t)(K * 3 + K * H) * 4;
  if ((size_t)4 * H * 4 > lds) lds = (size_t)4 * H * 4;
  compose_bwd_kernel<<<(unsigned)(H + K + (lp.out ? 1 : 0)), 256, lds, s>>>(dWc, W, E, H, K, dW, dE, lp);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ------------------------------------------------------------ logits backward
// dlog = q * (dq - <q, dq>) + scale * dlx,  dq = dq_dec + scale * dqx   (rows of the PCL layout)
__global__ void logits_bwd_kernel(const float* q, const float* dq_dec, const float* dqx, const float* dlx,
                                  const float* scale, int64_t R, int K, float* dlog) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const int L = ld4(K);  // pad channels: q = dq = dlx = 0 there, so dlog stays 0
  const float sc = scale ? *scale : 1.f;
  float s = 0.f;
  for (int k = 0; k < L; ++k) {
    const float dq = dq_dec[r * L + k] + sc * dqx[r * L + k];
    s = fmaf(q[r * L + k], dq, s);
  }
  for (int k = 0; k < L; ++k) {
    const float qk = q[r * L + k];
    const float dq = dq_dec[r * L + k] + sc * dqx[r * L + k];
    dlog[r * L + k] = qk * (dq - s) + sc * dlx[r * L + k];
  }
}

// The same, lane per channel (K <= 64): P = ld4(K) rounded up to a power of two lanes per row, 64 / P rows per
// wave, <q, dq> by xor shuffles inside the row's lanes (a fixed tree).  Loads and stores are whole rows, where
// the thread-per-row form above reads a row's channels with a 16 B-per-lane stride (cfg3 K = 32: 1.77 ms).
template <int P>
__global__ __launch_bounds__(256) void logits_bwd_lanes_kernel(const float* q, const float* dq_dec, const float* dqx,
                                                               const float* dlx, const float* scale, int64_t R, int L,
                                                               float* dlog) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = g / P;
  const int k = (int)(g - r * P);
  const bool on = r < R && k < L;
  const float sc = scale ? *scale : 1.f;
  const int64_t i = r * L + k;
  const float qk = on ? q[i] : 0.f;
  const float dq = on ? dq_dec[i] + sc * dqx[i] : 0.f;
  float s = qk * dq;
#pragma unroll
  for (int o = 1; o < P; o <<= 1) s += __shfl_xor(s, o);
  if (on) dlog[i] = qk * (dq - s) + sc * dlx[i];
}

int launch_logits_bwd(const float* q, const float* dq_dec, const float* dqx, const float* dlx, const float* scale,
                      int64_t R, int K, float* dlog, hipStream_t s) {
  if (R == 0) return VQHMM_OK;
  const int L = ld4(K);
  if (L <= 64) {
    const int P = L <= 4 ? 4 : L <= 8 ? 8 : L <= 16 ? 16 : L <= 32 ? 32 : 64;
    const unsigned nb = (unsigned)cdiv(R * P, 256);
    switch (P) {
      case 4: logits_bwd_lanes_kernel<4><<<nb, 256, 0, s>>>(q, dq_dec, dqx, dlx, scale, R, L, dlog); break;
      case 8: logits_bwd_lanes_kernel<8><<<nb, 256, 0, s>>>(q, dq_dec, dqx, dlx, scale, R, L, dlog); break;
      case 16: logits_bwd_lanes_kernel<16><<<nb, 256, 0, s>>>(q, dq_dec, dqx, dlx, scale, R, L, dlog); break;
      case 32: logits_bwd_lanes_kernel<32><<<nb, 256, 0, s>>>(q, dq_dec, dqx, dlx, scale, R, L, dlog); break;
      default: logits_bwd_lanes_kernel<64><<<nb, 256, 0, s>>>(q, dq_dec, dqx, dlx, scale, R, L, dlog); break;
    }
    VQHMM_LAUNCH_CHECK();
    return VQHMM_OK;
  }
  logits_bwd_kernel<<<(unsigned)cdiv(R, 256), 256, 0, s>>>(q, dq_dec, dqx, dlx, scale, R, K, dlog);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ------------------------------------------------------------ log_prior grad
// dlog_prior = dlp - softmax(log_prior) * sum(dlp),  dlp = c * sum_b q[b,:,0],  c = -beta/B (:71,:123,:131)
__device__ void log_prior_grad_body(const LogPriorGradArgs& a) {
  const int K = a.K;
  const float c = -a.beta / loss_norm_batch(a.norm, a.B);
  const float sc = a.scale ? *a.scale : 1.f;
  float m = -__builtin_inff();
  for (int k = 0; k < K; ++k) m = fmaxf(m, a.log_prior[k]);
  float se = 0.f;
  for (int k = 0; k < K; ++k) se += __expf(a.log_prior[k] - m);
  float tot = 0.f;
  for (int k = 0; k < K; ++k) tot += c * a.q0sum[k];
  for (int k = 0; k < K; ++k) a.out[k] = sc * (c * a.q0sum[k] - __expf(a.log_prior[k] - m) / se * tot);
}

// ------------------------------------------------------------ Prior backward (autograd of Prior.forward alone)
// log_A = log_softmax(lg) over each row i of a position's K x K logits (VQ_VAE_HMM_fixed.py:68-69):
//   dlg[i][j] = dA[i][j] - softmax(lg[i])_j * sum_j dA[i][j]   (thread per (PCL row, i); pad channels 0)
// and, by thread 0, log_pi = log_softmax(log_prior) (:71): dlp[k] = dlog_pi[k] - softmax(log_prior)_k sum dlog_pi
__global__ __launch_bounds__(256) void prior_lsm_bwd_kernel(const float* lg, const float* dA, int64_t R, int K,
                                                            float* dlg, const float* log_prior, const float* dlog_pi,
                                                            float* dlp) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g == 0 && dlp) {
    float m = -__builtin_inff();
    for (int k = 0; k < K; ++k) m = fmaxf(m, log_prior[k]);
    float se = 0.f, s = 0.f;
    for (int k = 0; k < K; ++k) {
      se += expf(log_prior[k] - m);
      s += dlog_pi ? dlog_pi[k] : 0.f;
    }
    for (int k = 0; k < K; ++k) dlp[k] = (dlog_pi ? dlog_pi[k] : 0.f) - expf(log_prior[k] - m) / se * s;
  }
  const int64_t r = g / K;
  const int i = (int)(g - r * K);
  if (r >= R) return;
  const int L = ld4(K * K);
  const float* lr = lg + r * L + i * K;
  const float* ar = dA + r * L + i * K;
  float m = -__builtin_inff();
  for (int j = 0; j < K; ++j) m = fmaxf(m, lr[j]);
  float se = 0.f, s = 0.f;
  for (int j = 0; j < K; ++j) {
    se += expf(lr[j] - m);
    s += ar[j];
  }
  for (int j = 0; j < K; ++j) dlg[r * L + i * K + j] = ar[j] - expf(lr[j] - m) / se * s;
  if (i == 0)
    for (int c = K * K; c < L; ++c) dlg[r * L + c] = 0.f;
}

int launch_prior_lsm_bwd(const float* lg, const float* dA, int64_t R, int K, float* dlg, const float* log_prior,
                         const float* dlog_pi, float* dlp, hipStream_t s) {
  const int64_t n = R * K > 0 ? R * K : 1;
  prior_lsm_bwd_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(lg, dA, R, K, dlg, log_prior, dlog_pi, dlp);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ------------------------------------------------------------ Adam
// torch.optim.Adam (no weight decay, no amsgrad), as its foreach/fused CUDA path computes it:
//   m = m + (1-b1)*(g-m);  v = b2*v + (1-b2)*g*g;
//   denom = sqrt(v)/sqrt(1-b2^t) + eps;  p = p - (lr/(1-b1^t)) * m/denom
// The step count t lives on the device so a captured HIP graph replays correct
// bias corrections, and the increment rides in the update's own launch: every
// workgroup reads t = (*step & 0xffffffff) + 1, then takes a ticket in the upper
// 32 bits; the last workgroup to do so (all reads are behind it) stores t with a
// zero ticket.  Between launches *step is the plain step count.  gmul scales the
// gradient first (1/world_size after a SUM all-reduce).
// Each thread takes float4 groups of all four buffers (vec: every pointer 16-byte aligned) strided over a
// grid of ~n / 1024 workgroups, and forms the bias corrections once (adam_load's expressions, so the same
// bits as the tail's fused update); the elements past the last whole group (and everything when !vec) go
// one per thread.  Few workgroups: few tickets on the step counter.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   double lr, double b1, double b2, double eps, int64_t* step,
                                                   float gmul, int vec) {
  const int64_t tn = (*step & 0xffffffffll) + 1;
  const AdamArgs a{p, m, v, step, lr, b1, b2, eps, gmul};
  AdamElem e;
  {
    const double t = (double)tn;
    e.step_size = (float)(a.lr / (1.0 - pow(a.b1, t)));
    e.bc2s = (float)sqrt(1.0 - pow(a.b2, t));
  }
  const int64_t stride = (int64_t)gridDim.x * 256, n4 = vec ? n / 4 : 0;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n4; j += stride) {
    const float4 gv = reinterpret_cast<const float4*>(g)[j], mv = reinterpret_cast<const float4*>(m)[j];
    const float4 vv = reinterpret_cast<const float4*>(v)[j], pv = reinterpret_cast<const float4*>(p)[j];
    const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, ma[4] = {mv.x, mv.y, mv.z, mv.w};
    const float va[4] = {vv.x, vv.y, vv.z, vv.w}, pa[4] = {pv.x, pv.y, pv.z, pv.w};
    float mo[4], vo[4], po[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e.m = ma[k]; e.v = va[k]; e.p = pa[k];
      const AdamOut o = adam_elem(a, ga[k], e);
      mo[k] = o.m; vo[k] = o.v; po[k] = o.p;
    }
    reinterpret_cast<float4*>(m)[j] = make_float4(mo[0], mo[1], mo[2], mo[3]);
    reinterpret_cast<float4*>(v)[j] = make_float4(vo[0], vo[1], vo[2], vo[3]);
    reinterpret_cast<float4*>(p)[j] = make_float4(po[0], po[1], po[2], po[3]);
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    e.m = m[i]; e.v = v[i]; e.p = p[i];
    adam_apply(a, i, g[i], e);
  }
  adam_ticket(step, tn);
}

// ------------------------------------------------------------ gradient clipping
// torch.nn.utils.clip_grad_norm_(params, max_norm) over the flat gradient (src/training/trainer.py:32):
//   g *= pre_scale;  total = ||g||_2;  g *= min(max_norm / (total + 1e-6), 1)
// One 1024-thread workgroup (the flat buffer is ~35k floats at cfg2): squares summed in double per
// thread, combined in a fixed order, then the same workgroup scales g in place.  The norm stays on the
// device (no host sync, graph-capturable).
__global__ __launch_bounds__(1024) void clip_grad_norm_kernel(float* g, int64_t n, float pre_scale, float max_norm,
                                                              float* total_out) {
  __shared__ double red[1024];
  __shared__ float coef;
  const int tid = threadIdx.x;
  double ss = 0.0;
  for (int64_t i = tid; i < n; i += 1024) {
    const float v = g[i] * pre_scale;
    ss += (double)v * (double)v;
  }
  red[tid] = ss;
  __syncthreads();
  for (int st = 512; st > 0; st >>= 1) {
    if (tid < st) red[tid] += red[tid + st];
    __syncthreads();
  }
  if (tid == 0) {
    const float total = (float)sqrt(red[0]);
    if (total_out) *total_out = total;
    coef = fminf(max_norm / (total + 1e-6f), 1.0f);
  }
  __syncthreads();
  const float c = coef * pre_scale;
  for (int64_t i = tid; i < n; i += 1024) g[i] *= c;
}

int launch_clip_grad_norm(float* g, int64_t n, float pre_scale, float max_norm, float* total_out, hipStream_t s) {
  clip_grad_norm_kernel<<<1, 1024, 0, s>>>(g, n, pre_scale, max_norm, total_out);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1, double beta2,
                double eps, int64_t* step, float gmul, hipStream_t s) {
  const auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const int vec = al(p) && al(g) && al(m) && al(v);
  const int64_t nb = std::min<int64_t>(std::max<int64_t>(cdiv(n, 1024), 1), 1024);  // >= 1: the step still advances
  adam_kernel<<<(unsigned)nb, 256, 0, s>>>(p, g, m, v, n, lr, beta1, beta2, eps, step, gmul, vec);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

}  // namespace vqhmm

namespace vqhmm {
__global__ void log_softmax_vec_kernel(const float* x, int K, float* out) {
  if (threadIdx.x != 0) return;
  float m = -__builtin_inff();
  for (int k = 0; k < K; ++k) m = fmaxf(m, x[k]);
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += __expf(x[k] - m);
  const float l = m + __logf(s);
  for (int k = 0; k < K; ++k) out[k] = x[k] - l;
}
int launch_log_softmax_vec(const float* x, int K, float* out, hipStream_t s) {
  log_softmax_vec_kernel<<<1, 64, 0, s>>>(x, K, out);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}
}  // namespace vqhmm

namespace vqhmm {
__device__ __forceinline__ void to_pcl_slot(const float* __restrict__ src, int C, int64_t B, int T, int64_t sc,
                                            int64_t st, float* __restrict__ dst, int64_t i) {  // i: float4 slot
  const int L4 = ld4(C) / 4;
  const int64_t R = B * (int64_t)(T + 2);
  if (i >= R * L4) return;
  int64_t r, b;
  int c0, t;
  bool valid;
  if (R * L4 <= 0x7fffffffll) {  // 32-bit index math (a 64-bit division is ~100 VALU ops per thread)
    const uint32_t i32 = (uint32_t)i, l4 = (uint32_t)L4, tp = (uint32_t)T + 2u;
    const uint32_t r32 = i32 / l4, b32 = r32 / tp;
    c0 = (int)(i32 - r32 * l4) * 4;
    t = (int)(r32 - b32 * tp) - 1;
    r = r32;
    b = b32;
    valid = t >= 0 && t < T;
  } else {
    r = i / L4;
    c0 = (int)(i - r * L4) * 4;
    valid = row_bt(r, R, T, b, t);
  }
  float e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    e[k] = (valid && c0 + k < C) ? src[b * (int64_t)C * T + (c0 + k) * sc + (int64_t)t * st] : 0.f;
  reinterpret_cast<float4*>(dst)[i] = make_float4(e[0], e[1], e[2], e[3]);
}
__global__ __launch_bounds__(256) void to_pcl_kernel(const float* __restrict__ src, int C, int64_t B, int T,
                                                     int64_t sc, int64_t st, float* __restrict__ dst) {
  to_pcl_slot(src, C, B, T, sc, st, dst, (int64_t)blockIdx.x * 256 + threadIdx.x);
}
// One 256-entry slice of a packed conv weight image (WImgJob, kernels.h).
__device__ __forceinline__ void wimg_slice(const WImgJob& j, int64_t i0) {
  const int NW = 16 * c2_nb(j.N), LDX = c2_ldx(j.Kc);
  const int64_t n_img = (int64_t)j.ks * NW * LDX;
  const int64_t i = i0 + threadIdx.x;
  if (i >= n_img) return;
  const int tap = (int)(i / (NW * LDX));
  const int rem = (int)(i - (int64_t)tap * NW * LDX);
  const int n = rem / LDX, c = rem - n * LDX;
  float v = 0.f;
  if (n < j.N && c < j.Kc) {
    // stored (a, b, tw): forward W[n][c][tap]; data gradient W[c][n][ks - 1 - tap]
    const int a = j.w_dgrad ? c : n, b = j.w_dgrad ? n : c, tw = j.w_dgrad ? j.ks - 1 - tap : tap;
    if (j.composed) return;  // Wc entries: written by the compose block of output channel a
    {
      const int inner = j.w_dgrad ? j.N : j.Kc;
      v = j.W[((int64_t)a * inner + b) * j.ks + tw];
    }
  }
  j.img[i] = v;
}

// One 256-entry slice of the cooperative head's weight image (PrologueArgs::himg, head_coop.hip CoopLds
// W2S | W1S): 16 * KB rows of W2 (ij >= K^2 zero) with stride TH + 4, then W1' = [W1 | b1 | 0] (TH x 8)
__device__ __forceinline__ void himg_slice(const PrologueArgs& a, int64_t i0) {
  const int KK = a.K * a.K, KB = (KK + 15) / 16, TH = a.hTH, LDW2 = TH + 4;
  const int64_t n2 = (int64_t)16 * KB * LDW2, i = i0 + threadIdx.x;
  if (i >= n2 + (int64_t)TH * 8) return;
  float v = 0.f;
  if (i < n2) {
    const int ij = (int)(i / LDW2), h = (int)(i - (int64_t)ij * LDW2);
    v = (ij < KK && h < TH) ? a.hW2[ij * TH + h] : 0.f;
  } else {
    const int k = (int)(i - n2), h = k >> 3, c = k & 7;
    v = c < a.U ? a.hW1[h * a.U + c] : (c == a.U ? a.hb1[h] : 0.f);
  }
  a.himg[i] = v;
}

// Step prologue in ONE launch (the step's first tiny pieces of work): blocks
// [0, nbx) convert x and [nbx, nbx + nbu) convert u to PCL (to_pcl_kernel), the next H
// blocks compose the decoder conv1 weight (compose_fwd_kernel), the rest pack the conv
// weight images (wimg_slice).
__global__ __launch_bounds__(256) void prologue_kernel(PrologueArgs a) {
  extern __shared__ float cs[];
  const unsigned bx = blockIdx.x;
  if (a.dbg) {  // timing experiment: skip the roles named by the bits
    const unsigned e1 = a.nbx + a.nbu, e2 = e1 + (unsigned)a.H, e3 = e2 + a.img_blk0[a.nimg], e4 = e3 + a.nbh;
    const int role = bx < e1 ? 1 : bx < e2 ? 2 : bx < e3 ? 4 : bx < e4 ? 8 : 16;
    if (a.dbg & role) return;
  }
  if (bx < a.nbx) {
    to_pcl_slot(a.x, a.D, a.B, a.T, a.xsc, a.xst, a.xp, (int64_t)bx * 256 + threadIdx.x);
  } else if (bx < a.nbx + a.nbu) {
    to_pcl_slot(a.u, a.U, a.B, a.T, a.usc, a.ust, a.up, (int64_t)(bx - a.nbx) * 256 + threadIdx.x);
  } else if (bx < a.nbx + a.nbu + (unsigned)a.H) {
    compose_fwd_block(a.W, a.E, a.H, a.K, a.Wc, (int)(bx - a.nbx - a.nbu), cs, a.wc_img_f, a.wc_img_d, a.Ecopy, a.Wcopy);
  } else if (bx < a.nbx + a.nbu + (unsigned)a.H + a.img_blk0[a.nimg]) {
    const unsigned ib = bx - a.nbx - a.nbu - (unsigned)a.H;
    int j = 0;
    while (j + 1 < a.nimg && ib >= a.img_blk0[j + 1]) ++j;
    wimg_slice(a.img[j], (int64_t)(ib - a.img_blk0[j]) * 256);
  } else if (bx < a.nbx + a.nbu + (unsigned)a.H + a.img_blk0[a.nimg] + a.nbh) {
    himg_slice(a, (int64_t)(bx - a.nbx - a.nbu - (unsigned)a.H - a.img_blk0[a.nimg]) * 256);
  } else {  // the batch's valid count mask.sum() (VQ_VAE_HMM_fixed.py:111,:120), fixed order
    __shared__ unsigned long long cred[256];
    unsigned long long c = 0;
    for (int64_t b = threadIdx.x; b < a.B; b += 256) {
      const int64_t L = a.lengths[b];
      c += (unsigned long long)(L <= 0 ? 0 : (L < a.T ? L : a.T));
    }
    cred[threadIdx.x] = c;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if ((int)threadIdx.x < st) cred[threadIdx.x] += cred[threadIdx.x + st];
      __syncthreads();
    }
    if (threadIdx.x == 0) *a.cnt = (int64_t)cred[0];
  }
}
// profiling build only (VQHMM_PRO_EMPTY / VQHMM_TAIL_EMPTY = n): n empty launches (256 workgroups, no LDS)
// right before the prologue / the tail, to attribute what a launch costs after the one before it
// (tools/gpu_launch_attr.sh)
__global__ __launch_bounds__(256) void prof_empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}
static void prof_empties(const char* name, hipStream_t s) {
  const char* e = VQHMM_PROF_ENV(name);
  const int n = e ? atoi(e) : 0;
  for (int k = 0; k < n; ++k) prof_empty_kernel<<<256, 256, 0, s>>>(nullptr);
}

int launch_prologue(PrologueArgs a, hipStream_t s) {
  prof_empties("VQHMM_PRO_EMPTY", s);
  {
    static const char* dbg = VQHMM_PROF_ENV("VQHMM_PRO_DBG");
    a.dbg = dbg ? atoi(dbg) : 0;
  }
  const int64_t R = a.B * (int64_t)(a.T + 2);
  a.nbx = (unsigned)cdiv(R * (ld4(a.D) / 4), 256);
  a.nbu = (unsigned)cdiv(R * (ld4(a.U) / 4), 256);
  if (a.nimg < 0 || a.nimg > MAX_WIMG) return VQHMM_EINVAL;
  a.img_blk0[0] = 0;
  for (int j = 0; j < a.nimg; ++j)
    a.img_blk0[j + 1] = a.img_blk0[j] + (unsigned)cdiv(c2_image_floats(a.img[j].N, a.img[j].Kc, a.img[j].ks), 256);
  a.nbh = a.himg ? (unsigned)cdiv(head_coop_image_floats(a.K, a.hTH), 256) : 0u;
  const size_t lds = (size_t)(a.H * 3 + a.K * a.H) * 4;
  prologue_kernel<<<a.nbx + a.nbu + (unsigned)a.H + a.img_blk0[a.nimg] + a.nbh + (a.cnt ? 1u : 0u), 256, lds, s>>>(a);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}
int launch_to_pcl(const float* src, int C, int64_t B, int T, int64_t sc, int64_t st, float* dst, hipStream_t s) {
  const int64_t n = B * (int64_t)(T + 2) * (ld4(C) / 4);
  if (n == 0) return VQHMM_OK;
  to_pcl_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(src, C, B, T, sc, st, dst);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}
}  // namespace vqhmm

// ------------------------------------------------------------ data step
// Device-side RandomChunkDataset.__getitem__ + collate_fn (VQ_VAE_HMM_fixed.py:
// 25-29, 164-179): out (B, C, Tm) with
//   out[i, c, t] = t < L_i ? src[base_i + c * n_i + s_i + t] : 0,
// meta_i = {base_i, n_i, s_i, L_i}: sample i is columns [s_i, s_i + L_i) of a
// row-major (C, n_i) sequence stored at element base_i of src.  Consecutive
// threads walk t, so reads and writes are contiguous runs.
namespace vqhmm {
__global__ __launch_bounds__(256) void gather_chunks_kernel(const float* __restrict__ src,
                                                            const int64_t* __restrict__ meta, int64_t B, int C,
                                                            int Tm, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C * (int64_t)Tm) return;
  const int t = (int)(i % Tm);
  const int64_t r = i / Tm;
  const int c = (int)(r % C);
  const int64_t* m = meta + (r / C) * 4;
  out[i] = t < m[3] ? src[m[0] + c * m[1] + m[2] + t] : 0.f;
}

int launch_gather_chunks(const float* src, const int64_t* meta, int64_t B, int64_t C, int64_t Tm, float* out,
                         hipStream_t s) {
  const int64_t n = B * C * Tm;
  if (n == 0) return VQHMM_OK;
  gather_chunks_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(src, meta, B, (int)C, (int)Tm, out);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}

// ------------------------------------------------------------ hard regimes
// idx[b, t] = first argmax_k q[b, k, t] of a CF (B, K, T) tensor, torch.argmax's rule
// (NaN counts as the maximum, lowest index on ties): regime_probs.argmax(dim=1) of
// backtesting.py:154-155 / VQ_VAE+HMM.ipynb:830.  Consecutive threads walk t (coalesced).
__global__ __launch_bounds__(256) void argmax_cf_kernel(const float* __restrict__ q, int64_t B, int K, int64_t T,
                                                        int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B * T) return;
  const int64_t b = i / T, t = i - b * T;
  const float* col = q + b * K * T + t;
  float bq = col[0];
  int bi = 0;
  for (int k = 1; k < K; ++k) {
    const float v = col[(int64_t)k * T];
    if (argmax_beats(v, k, bq, bi)) { bq = v; bi = k; }
  }
  idx[i] = bi;
}

int launch_argmax_cf(const float* q, int64_t B, int64_t K, int64_t T, int32_t* idx, hipStream_t s) {
  const int64_t n = B * T;
  if (n == 0) return VQHMM_OK;
  argmax_cf_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(q, B, (int)K, T, idx);
  VQHMM_LAUNCH_CHECK();
  return VQHMM_OK;
}
}  // namespace vqhmm
