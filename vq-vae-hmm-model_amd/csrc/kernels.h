// Internal interface between the kernel translation units and the executor
// (api.hip).  Not part of the public C-ABI (include/vqhmm.h).
#pragma once
#include "common.h"

namespace vqhmm {

// All PCL tensors below have row stride ld4(channels) with zero pad channels.
struct ConvArgs {
  const float* src;  // input activations
  int src_cf;        // 1: CF (B, Kc, T) (generic kernel only); 0: PCL (R, ld4(Kc))
  int Kc;            // input channels (GEMM K per tap)
  int64_t R;
  int T;
  int ks;            // 1 or 3
  const float* W;
  int w_dgrad;       // 0: W is (N, Kc, ks); 1: W is (Kc, N, ks) used transposed + flipped
  const float* Wimg; // conv2_kernel only: W already packed in its LDS layout (WImgJob), or null
  const float* bias; // (N) or null
  const float* scale;// device scalar multiplying the accumulator, or null
  int N;             // output channels
  int act;           // 0 none, 1 relu, 2 multiply by (aux > 0)
  const float* aux;  // PCL (R, ld4(N)) for act == 2
  float* out;        // PCL (R, ld4(N)) or null
  float* out_cf;     // CF (B, N, T) or null
  // fused 1x1 tail on the activated output (requires N <= BN)
  const float* tW;   // (C2, N)
  const float* tb;   // (C2)
  int C2;
  float* t_out;      // PCL (R, ld4(C2))
  float* t_cf0;      // CF, channels [0, t_split)
  float* t_cf1;      // CF, channels [t_split, C2)
  int t_split;
  float* q_out;      // PCL softmax of the tail
  float* q_cf;       // CF softmax of the tail
  int32_t* reg_out;  // (B, T) first-index argmax over channels of that softmax (torch.argmax rule)
  // act == 3 (conv2 only, N <= 4; act == 4: N <= 8): the output y = dL/dq of the decoder path is also
  // pushed through the softmax backward (logits_bwd_kernel's formula):
  // lb_dlog = q * (dq - <q, dq>) + scale * lb_dlx,  dq = y + scale * lb_dqx
  const float* lb_q;
  const float* lb_dqx;
  const float* lb_dlx;
  const float* lb_scale;
  float* lb_dlog;
  // ... and, when lb_dh is set (ld4(lb_C) % 16 == 0), to_logits' dgrad with the ReLU mask of its
  // input: lb_dh = (lb_h > 0) * (lb_W^T @ lb_dlog), lb_W the (N, lb_C) to_logits weight
  const float* lb_W;
  const float* lb_h;
  float* lb_dh;
  int lb_C;
  int pipe;          // conv2 kernels: software-pipelined operand reads (set by the launcher)
  // fused front conv (conv2f only, f_Wimg set): src is the INPUT of a k=3 ReLU conv f_Kc -> Kc
  // (f_Kc <= 16, Kc <= 64; weights packed in conv2w<4, 1, 3>'s image layout), whose output rows
  // are written to f_out (PCL, ld4(Kc)) and feed this conv from LDS, never re-read from HBM
  // (or, f_ks = 1 / f_act = 2 with this conv's act = 2: a 1x1 data-gradient front with the ReLU
  // mask f_aux, scaled by *f_scale, feeding a masked k=3 data gradient)
  int f_Kc, f_ks, f_act;
  const float* f_Wimg;
  const float* f_bias;
  const float* f_aux;
  const float* f_scale;
  float* f_out;
  int prof;          // conv2 kernels: phase stamps (prof.h, VQHMM_CONV_PROF; set by the launcher)
};

// Loss normalisers of compute_loss (VQ_VAE_HMM_fixed.py:120 mask.sum()*C, :131/:135 B).
// norm == null: the batch's own valid count and B.  norm = device int64 {valid_count, batch}:
// the normalisers of a larger global batch this batch is a shard of, so per-shard losses and
// gradients SUM (all-reduce) to exactly the global batch's (data parallel over ragged batches).
__device__ __forceinline__ float loss_norm_batch(const int64_t* norm, int64_t B) {
  return norm ? (float)norm[1] : (float)B;
}

// finalize_loss: loss = recon + beta*(prior - entropy) (VQ_VAE_HMM_fixed.py:137) from the head's
// per-workgroup partials part[nblk][4] = recon_sum, init_sum, trans_sum, ent_sum; run by the 256
// threads of ONE workgroup; red = 5*256 doubles of LDS.
// cnt (nullable): the batch's valid count already reduced on the device (the prologue's), used
// instead of a pass over lengths when norm is null.
__device__ inline void finalize_loss_block(const double* part, int nblk, const int64_t* lengths, const int64_t* norm,
                                           int64_t B, int T, int D, float beta, float* loss, double* accum,
                                           float* pieces, double* red, const int64_t* cnt = nullptr) {
  const int tid = threadIdx.x;
  double v[5] = {0, 0, 0, 0, 0};
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int i = tid; i < nblk; i += 256)
    for (int k = 0; k < 4; ++k) v[k] += part[i * 4 + k];
  if (!norm && cnt && tid == 0) v[4] = (double)*cnt;
#pragma unroll 8  // independent load -> store iterations: keep 8 loads in flight
  for (int64_t b = tid; !norm && !cnt && b < B; b += 256) {
    const int64_t L = lengths[b];
    v[4] += (double)(L <= 0 ? 0 : (L < T ? L : T));
  }
  for (int k = 0; k < 5; ++k) red[k * 256 + tid] = v[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st)
      for (int k = 0; k < 5; ++k) red[k * 256 + tid] += red[k * 256 + tid + st];
    __syncthreads();
  }
  if (tid == 0) {
    const double cnt = norm ? (double)norm[0] : red[4 * 256];
    const double Bn = norm ? (double)norm[1] : (double)B;
    const float ncount = fmaxf((float)(cnt * D), 1.0f);
    const float recon = (float)red[0] / ncount;
    const float prior = -(float)((red[1 * 256] + red[2 * 256]) / Bn);
    const float ent = (float)(red[3 * 256] / Bn);
    const float l = recon + beta * (prior - ent);
    *loss = l;
    if (accum) *accum += (double)l;
    if (pieces) { pieces[0] = recon; pieces[1] = prior; pieces[2] = ent; }
  }
}

struct WgradArgs {
  const float* dy;   // PCL (R, ld4(N)) output gradient (pad rows zero)
  const float* x;    // layer input: PCL (R, ld4(C)) or CF (B, C, T) (generic kernel only)
  int x_cf;
  int64_t R;
  int T;
  int N, C, ks;
  int64_t rows_per_chunk;  // multiple of 64
  float* slab;       // [nchunks][N][C][ks]
  float* bias_slab;  // [nchunks][N] or null
  int ld_dy;         // dY row stride in floats (grouped body; a slice of a wider dY), 0: ld4(N)
  // the composed decoder conv1 (grouped launch; N = H outputs o, C = K inputs k, k = 3, N*C*3 <= 1536):
  // each chunk also writes its share of the embedding gradient,
  //   cmp_slab[chunk][k][h] = sum_{o, tap} dWc_chunk[o][k][tap] * cmpW[o][h][tap],
  // so the backward tail needs no reduced dWc before it can form dE (no cross-workgroup wait)
  const float* cmpW;  // decoder.conv1.weight (H, H, 3), or null
  float* cmp_slab;    // [nchunks][K][H]
};

struct HeadArgs {
  int dbg;               // head profiling switch (profiling build, VQHMM_HEAD_DBG bits; 16: phase stamps);
                         // 0 in every product launch
  int64_t B;
  int T;
  int64_t R;
  int D, K, U, TH;
  const float* x;        // PCL (R, ld4(D))  (x converted once per step)
  const float* u;        // PCL (R, ld4(U))
  const int64_t* lengths;
  const float* par;      // PCL (R, ld4(2D)): mu | logvar
  const float* logits;   // PCL (R, ld4(K))
  const float* q;        // PCL (R, ld4(K))
  const float* W1;       // (TH, U)
  const float* b1;       // (TH)
  const float* W2;       // (K*K, TH)
  const float* b2;       // (K*K)
  const float* log_prior;// (K)
  float beta;
  const int64_t* norm;   // null, or device {valid_count, batch}: global normalisers (see loss_norm)
  const int64_t* cnt_in; // without norm: the batch's valid count if the prologue already wrote it (else counted)
  int need_grad;
  float* dpar;           // PCL (R, ld4(2D))
  float* dqx;            // PCL (R, ld4(K))  dL/dq from the prior term
  float* dlx;            // PCL (R, ld4(K))  dL/dlogits from the entropy term
  double* part;          // [gridDim.x][4]: recon_sum, init_sum, trans_sum, ent_sum
  float* slab_W1;        // [grid][TH*U]
  float* slab_b1;        // [grid][TH]
  float* slab_W2;        // [grid][K*K*TH]
  float* slab_b2;        // [grid][K*K]
  float* slab_q0;        // [grid][K]  sum_b q[b, :, 0]
  const float* himg;     // head_coop: the prologue's image of the Prior MLP weights (LDS DMA), or null
  int64_t ntiles;
};

struct PriorArgs {
  int64_t B;
  int T, K, U, TH;
  const float* u;
  int64_t u_sc, u_st;
  const float *W1, *b1, *W2, *b2;
  float* log_A;  // (B, T, K, K)
};

struct LogPriorGradArgs {  // log_prior gradient (misc.hip log_prior_grad_body); out == null: skipped
  const float* q0sum;
  const float* log_prior;
  int K;
  float beta;
  const int64_t* norm;
  int64_t B;
  const float* scale;
  float* out;
};
struct SlabSeg {
  const float* slab;   // [nchunks][len] ([nchunks][cmpH * cmpK * 3] for a composed segment)
  float* out;          // [len]
  const float* scale;  // device scalar or null
  int64_t nchunks, len;
  // composed segment (cmpE set): out[j], j = (o * H + h) * 3 + tap, is the decoder conv1 weight gradient
  // dW[o][h][tap] = sum_k dWc[o][k][tap] E[k][h] (VQ_VAE_HMM_fixed.py:83-85 folded), where each
  // block reduces the dWc slab columns of its own o rows itself
  const float* cmpE;   // (K, H): the embedding as this step's forward used it
  int cmpH, cmpK;
  // trO > 0: a conv weight (trO, trC, 3) whose rows are stored output-fastest, column (c * 3 + tap) * trO + o
  // holding out[(o * trC + c) * 3 + tap] (the backward strip's 64-wide layers)
  int trO, trC;
};
__host__ __device__ inline int64_t seg_out_index(const SlabSeg& sg, int64_t col) {
  if (sg.trO == 0) return col;
  const int64_t ct = col / sg.trO, c = ct / 3;
  return ((col - ct * sg.trO) * sg.trC + c) * 3 + (ct - 3 * c);
}
// largest dWc column span one 64-column block of a composed segment reduces (block_reduce_cols' 256)
__host__ __device__ inline int64_t composed_block_cols(int H, int K) { return (int64_t)(2 + 62 / (3 * H)) * 3 * K; }

int launch_vq_argmin(const float* z, int64_t B, int64_t Dv, int64_t T, const float* cb, int64_t K, int32_t* idx,
                     float* dmin, hipStream_t s);
// quantize (pseudocode.txt:12-18): argmin + z_q gather + straight-through value + sum (z - z_q)^2
size_t vq_quantize_ws_bytes(int64_t B, int64_t Dv, int64_t T, int64_t K);
int launch_vq_quantize(const float* z, int64_t B, int64_t Dv, int64_t T, const float* cb, int64_t K, int32_t* idx,
                       float* zq_st, double* sse, void* ws, size_t ws_bytes, hipStream_t s);
int launch_conv(const ConvArgs& a, hipStream_t s);
// wide convolutions and weight gradients on the f32 MFMA (convbig.hip): Kc % 16 == 0, N % 4 == 0, PCL in / out
bool convbig_supported(const ConvArgs& a);
int launch_convbig(const ConvArgs& a, hipStream_t s);
bool conv2_supported(const ConvArgs& a);
// front conv + this conv in one launch (conv2.hip conv2f_kernel; ConvArgs::f_*)
bool conv2_fused_supported(const ConvArgs& a);
int launch_conv2_fused(const ConvArgs& a, hipStream_t s);
// dec_conv1 dgrad (+ logits backward, to_logits dgrad: f) -> enc_conv2 dgrad (a) in one launch
bool conv2_bwd_pair_supported(const ConvArgs& a, const ConvArgs& f);
int launch_conv2_bwd_pair(const ConvArgs& a, const ConvArgs& f, hipStream_t s);
// Packed weight image of a conv2_kernel launch: img[(tap*NW + n)*LDX + c] = Weff(n, c, tap)
// (zero past N / Kc), NW = 16*NB and LDX = 16*KCP + 4 for the launch's (NB, KCP) (c2_nb / c2_kcp).
// Built once per step (prologue), so every workgroup stages its weights with float4 copies.
// composed = 1: the logical weight is the decoder's folded conv1, Wc[o][k][tap] =
// sum_h W[o][h][tap] E[k][h] (W (H,H,3), E (K,H)); the job writes only the image's zero
// padding, the prologue's compose blocks write the Wc entries (PrologueArgs::wc_img_*).
struct WImgJob {
  const float* W;
  const float* E;  // composed only
  int composed, H; // composed only: H = reduction length of the fold
  int w_dgrad, N, Kc, ks;
  float* img;
};
__host__ __device__ inline int c2_nb(int N) { return N <= 16 ? 1 : N <= 32 ? 2 : 4; }
__host__ __device__ inline int c2_kcp(int Kc) { return Kc <= 16 ? 1 : Kc <= 32 ? 2 : 4; }
// LDS row stride of conv2_kernel's W / X tiles: 16*KCP + 8 floats makes the ds_read_b128 operand reads
// (lane (lg4, l16) -> row l16, float4 lg4) bank-conflict free in all four 16-lane groups (+4 was 2-way)
__host__ __device__ inline int c2_ldx(int Kc) { return 16 * c2_kcp(Kc) + 8; }
__host__ __device__ inline int64_t c2_image_floats(int N, int Kc, int ks) {
  return (int64_t)ks * 16 * c2_nb(N) * c2_ldx(Kc);
}
int launch_conv2(const ConvArgs& a, hipStream_t s);
// Forward strip kernel (strip.hip): enc_conv1 -> enc_conv2 + to_logits + softmax -> composed dec_conv1
// -> dec_conv2 + to_params in ONE launch over 128-row strips, the activations between layers in LDS
// (the four ConvArgs of the separate launches; packed-tap fronts, H = 64, H2 <= 32, K <= 4, 2D <= 16)
bool strip_fwd_supported(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2);
// h (nullable): the ELBO head fused after the decoder (strip_head_supported: K <= 4, U <= 4, TH in {64, 128},
// D <= 8); its slabs / loss partials have strip_fwd_grid(R) rows
bool strip_head_supported(const HeadArgs& h);
int strip_fwd_grid(int64_t R);
int launch_strip_fwd(const ConvArgs& e1, const ConvArgs& e2, const ConvArgs& d1, const ConvArgs& d2, const HeadArgs* h,
                     hipStream_t s);
// Backward strip kernel (strip.hip): to_params dgrad -> dec_conv2 dgrad -> composed dec_conv1 dgrad +
// softmax backward + to_logits dgrad -> enc_conv2 dgrad in ONE launch (the four ConvArgs of those launches;
// f = dec_conv1's ACT 3 args with lb_dh; H = 64, H2 in (16, 32], K <= 4, 2D <= 16)
bool strip_bwd_supported(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2);
int launch_strip_bwd(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2, hipStream_t s);
// The backward strip with the six weight gradients folded in (strip_bwdw.hip): the same four ConvArgs plus
// the X operands the chain does not carry and one slab row per workgroup for every layer (S_W_PAR .. S_W_ENC1
// order, wgrad2's [chunk][N][C][ks] / [chunk][N] layouts; chunk = workgroup, strip_bwdw_grid(R) of them);
// D <= 5, K <= 4 (packed-tap enc_conv1 / dec_conv1 weight gradients)
struct StripWgradArgs {
  const float* x;        // PCL (R, ld4(D)): enc_conv1's input
  const float* cmpW;     // decoder.conv1.weight (H, H, 3): the composed layer's dE shares
  float* slab[6];
  float* bslab[6];
  float* cslab;          // [grid][K][H]
  int D, K, H2;
  int64_t* step_inc;     // non-null: workgroup 0 advances the fused tail's Adam step counter
  int store;             // 1: also store dg2 / dg1 / dh1 (the separate launches' dY; never needed by the step)
};
bool strip_bwdw_supported(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2, int D);
int strip_bwdw_own(int64_t R);
int strip_bwdw_grid(int64_t R);
int launch_strip_bwdw(const ConvArgs& pd, const ConvArgs& d2, const ConvArgs& f, const ConvArgs& e2,
                      const StripWgradArgs& w, hipStream_t s);
// phase stamps of the last profiled launch (prof.h): strip.hip (VQHMM_STRIP_PROF), conv2.hip (VQHMM_CONV_PROF)
int strip_prof_copy(uint64_t* out, int64_t n);
int conv2_prof_copy(uint64_t* out, int64_t n);
int head_prof_copy(uint64_t* out, int64_t n);  // head_coop.hip (VQHMM_HEAD_PROF)
int bwdw_prof_copy(uint64_t* out, int64_t n);  // strip_bwdw.hip (VQHMM_STRIP_PROF)
int launch_wgrad(const WgradArgs& a, hipStream_t s);
bool wgradbig_supported(const WgradArgs& a);
int64_t wgradbig_rows(int64_t R, int N, int C);
int launch_wgradbig(const WgradArgs& a, hipStream_t s);
int64_t wgrad_chunks(int64_t R, int64_t tiles);
bool wgrad2_supported(const WgradArgs& a);
int64_t wgrad2_rows(int64_t R, int N, int C, int ks);
int launch_wgrad2(const WgradArgs& a, hipStream_t s);
// A step's weight gradients as ONE launch (wgrad2.hip): job j's chunks are workgroups
// [blk0[j], blk0[j+1]); every job must be wgrad2_group_supported.
constexpr int MAX_WJOBS = 8;
struct WgradGroup {
  WgradArgs job[MAX_WJOBS];
  int variant[MAX_WJOBS], wn[MAX_WJOBS], wc[MAX_WJOBS];
  int64_t blk0[MAX_WJOBS + 1];
  int njobs;
  int64_t* step_inc;  // non-null: the Adam step counter this backward's tail applies; workgroup 0 advances it
};
bool wgrad2_group_supported(const WgradArgs& a);
// a grouped job's rows per chunk (a multiple of its stage rows: 64, or 192 for the small outputs)
int64_t wgrad2_group_rows(int64_t rows, int N, int C, int ks);
int launch_wgrad2_group(const WgradArgs* jobs, int n, hipStream_t s, int64_t* step_inc = nullptr);
// Staged ELBO head (head_staged.hip): shapes the fused heads do not cover.
struct StagedHeadArgs {
  int64_t B;
  int T;
  int64_t R;
  int D, K;
  const float *x, *par, *logits, *q;  // PCL
  const int64_t* lengths;
  const float* log_prior;
  float* log_pi;                      // (K) scratch
  float* lgA;                         // PCL (R, ld4(K*K)): transition logits in, d logits out
  float *nx, *dqc, *trw;              // PCL (R, ld4(K)) x2, (R)
  float beta;
  const int64_t* norm;                // null, or device {valid_count, batch} (see loss_norm)
  int need_grad;
  float *dpar, *dlx, *dqx;
  double* part;                       // [l2grid][4]
  float* q0;                          // (K)
};
bool staged_head_supported(int K);
bool fused_head_supported(const HeadArgs& a);
int launch_staged_head(const StagedHeadArgs& a, int l2grid, hipStream_t s);

int head_grid(int64_t R);
bool head_mfma_supported(const HeadArgs& a);
int launch_head_mfma(const HeadArgs& a, int grid, hipStream_t s);
// workgroup-cooperative MFMA head (head_coop.hip): K <= 8, U <= 4, TH in {64, 128, 256}, D <= 16; its
// grid / slab count
bool head_coop_supported(const HeadArgs& a);
// floats of the head image the prologue builds for elbo_head_coop_kernel (PrologueArgs::himg)
int64_t head_coop_image_floats(int K, int TH);
int head_coop_grid(int64_t R, int K);
int launch_head_coop(const HeadArgs& a, int grid, hipStream_t s);
// its pipelined form for K <= 4, TH = 128 (one 12-wave workgroup per CU: MFMA waves + row waves)
bool head_pipe_supported(const HeadArgs& a);
int head_pipe_grid(int64_t R);
int launch_head_pipe(const HeadArgs& a, int grid, hipStream_t s);
int launch_head(const HeadArgs& a, int grid, hipStream_t s);
int launch_prior_fwd(const PriorArgs& p, hipStream_t s);
// Prior.forward on MFMA (prior.hip): K*K <= 64, U <= 4, TH in {64, 128, 256}
bool prior_mfma_supported(const PriorArgs& p);
int launch_prior_mfma(const PriorArgs& p, hipStream_t s);
// Fused Prior.forward -> Viterbi (prior_viterbi.hip): K <= 8, U <= 4, TH in {64, 128, 256};
// log_pi on the device, ws = viterbi_ws_bytes(B, T, K); p.log_A unused
bool prior_viterbi_supported(const PriorArgs& p);
int launch_prior_viterbi(const PriorArgs& p, const float* log_pi, const float* em, const int64_t* lengths,
                         int32_t* path, float* score, void* ws, size_t ws_bytes, hipStream_t s);
// Backward tail (misc.hip grad_tail_kernel), ONE launch: every gradient segment's slabs summed in a
// fixed chunk order (deterministic, no atomics) and scaled; one extra workgroup reduces the q0 slab
// and writes the log_prior gradient.
constexpr int MAX_SEGS = 24;
struct TailArgs {
  SlabSeg s[MAX_SEGS];
  int64_t blk_start[MAX_SEGS + 1];  // set by launch_grad_tail
  int nseg;
  const float* q0slab;   // [q0chunks][K]: sum_b q[b, :, 0] partials (log_prior gradient), or null
  int64_t q0chunks;
  LogPriorGradArgs lp;   // q0sum unused (the tail block reduces q0slab itself)
  // loss finalize deferred from the forward (fin_loss set): one more workgroup runs
  // finalize_loss_block on the head's partials with the prologue's valid count
  const double* fin_part;
  int fin_nblk;
  const int64_t* fin_cnt;
  int64_t fin_B;
  int fin_T, fin_D;
  float* fin_loss;
  double* fin_accum;
  float* fin_pieces;
  int dbg;  // profiling build only (VQHMM_TAIL_DBG): 1 skip segment reductions, 2 log_prior, 4 loss, 8 Adam
};
// torch.optim.Adam over the flat buffers (misc.hip adam_kernel / compose_adam_kernel)
struct AdamArgs {
  float* p;
  float* m;
  float* v;
  int64_t* step;         // device step counter (+ completion ticket in the upper 32 bits)
  double lr, b1, b2, eps;
  float gmul;
};
// The non-grouped path's composed decoder conv1 (a launch after grad_tail reduced dWc):
// dW[o][h][tap] = sum_k dWc[o][k][tap] E[k][h] and dE[k][h] = sum_{o,tap} dWc[o][k][tap] W[o][h][tap]
// written into g, then (compose_adam) every element's Adam update; E, W: the prologue's copies, since
// that launch updates the parameters.
struct ComposeAdamArgs {
  const float* dWc;      // (H, K, 3) reduced
  const float* Ecopy;    // (K, H)
  const float* Wcopy;    // (H, H, 3)
  int H, K;
  float* g;              // flat gradient
  int64_t n;             // elements
  int64_t off_w, off_e;  // element offsets of decoder.conv1.weight and decoder.embeddings.weight
  AdamArgs adam;
};
int launch_compose_adam(const ComposeAdamArgs& a, hipStream_t s);
// The backward tail in ONE launch (misc.hip tail_kernel): grad_tail's blocks, each (adam != null) then
// applying Adam to the columns it has just reduced; the composed segment's blocks form dW themselves,
// so no block waits for another.  g = the flat gradient buffer the segments write into.  With adam, an
// earlier launch of the same step must have advanced *adam->step (launch_wgrad2_group's step_inc).
int launch_tail(TailArgs& ta, const AdamArgs* adam, const float* g, hipStream_t s);
int launch_grad_tail(TailArgs& a, hipStream_t s);
int launch_finalize_loss(const double* part, int nblk, const int64_t* lengths, const int64_t* norm, int64_t B, int T,
                         int D, float beta, float* loss, double* accum, float* pieces, hipStream_t s);
int launch_compose_fwd(const float* W, const float* E, int H, int K, float* Wc, hipStream_t s);
int launch_compose_bwd(const float* dWc, const float* W, const float* E, int H, int K, float* dW, float* dE,
                       const LogPriorGradArgs& lp, hipStream_t s);
// Prior.forward's log_softmax backward (rows of K of each PCL row's K*K logits) + log_pi's (misc.hip)
int launch_prior_lsm_bwd(const float* lg, const float* dA, int64_t R, int K, float* dlg, const float* log_prior,
                         const float* dlog_pi, float* dlp, hipStream_t s);
int launch_logits_bwd(const float* q, const float* dq_dec, const float* dqx, const float* dlx, const float* scale,
                      int64_t R, int K, float* dlog, hipStream_t s);
// CF / (B,T,C) tensor -> PCL (R, ld4(C)) with zero pad rows / channels:
// dst[b*(T+2)+1+t][c] = src[b*C*T + c*sc + t*st]
int launch_to_pcl(const float* src, int C, int64_t B, int T, int64_t sc, int64_t st, float* dst, hipStream_t s);
constexpr int MAX_WIMG = 12;
struct PrologueArgs {  // step prologue: x, u -> PCL, the composed decoder conv1 weight and the conv weight images
  const float* x; int D; int64_t xsc, xst; float* xp;
  const float* u; int U; int64_t usc, ust; float* up;
  int64_t B; int T;
  const float* W; const float* E; int H, K; float* Wc;
  WImgJob img[MAX_WIMG];
  int nimg;
  float* wc_img_f;  // images of the composed decoder conv1 (forward / data gradient), or null
  float* wc_img_d;
  float* Ecopy;     // (K, H) / (H, H, 3) copies of the embedding and decoder.conv1's weight for the
  float* Wcopy;     // launches that read them while Adam updates the parameters, or null
  const int64_t* lengths;  // with cnt: the last block writes the batch's valid count
  int64_t* cnt;            // (sum_b min(max(L_b, 0), T)) for a loss finalized in the backward, or null
  // the cooperative head's Prior MLP weights in its LDS layout (head_coop_image_floats), or himg = null:
  // [W2 rows ij (16 * ceil(K^2 / 16) of them, zero past K^2) x (TH + 4) | W1' = [W1 | b1 | 0] (TH x 8)]
  const float *hW1, *hb1, *hW2;
  int hTH;
  float* himg;
  unsigned nbh;                     // set by launch_prologue
  unsigned nbx, nbu;                // set by launch_prologue
  unsigned img_blk0[MAX_WIMG + 1];  // set by launch_prologue: first block of each image
  int dbg;  // profiling build only (VQHMM_PRO_DBG): skip block roles 1 x/u, 2 compose, 4 images, 8 head image, 16 count
};
int launch_prologue(PrologueArgs a, hipStream_t s);
int launch_gather_chunks(const float* src, const int64_t* meta, int64_t B, int64_t C, int64_t Tm, float* out,
                         hipStream_t s);
int launch_log_softmax_vec(const float* x, int K, float* out, hipStream_t s);
int launch_argmax_cf(const float* q, int64_t B, int64_t K, int64_t T, int32_t* idx, hipStream_t s);
size_t viterbi_ws_bytes(int64_t B, int64_t T, int64_t K);
// K > 32 (<= 4096): one workgroup per sequence, thread = states j, j + 256, .. (hmm_generic.hip)
bool hmm_generic_supported(int64_t K);
size_t hmm_generic_viterbi_ws_bytes(int64_t B, int64_t T, int64_t K);
size_t hmm_generic_fwdbwd_ws_bytes(int64_t B, int64_t T, int64_t K);
int launch_viterbi_generic(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                           int64_t B, int64_t T, int64_t K, int32_t* path, float* score, void* ws, hipStream_t s);
int launch_fwdbwd_generic(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                          int64_t B, int64_t T, int64_t K, float* gamma, float* logZ, void* ws, hipStream_t s);
// K in (8, 32]: one sequence per wave (hmm_wide.hip)
size_t viterbi_wide_ws_bytes(int64_t B, int64_t T);
int launch_viterbi_wide(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                        int64_t T, int64_t K, int32_t* path, float* score, void* ws, hipStream_t s);
int launch_fwdbwd_wide(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                       int64_t T, int64_t K, float* gamma, float* logZ, float* ws, hipStream_t s);
size_t fwdbwd_ws_bytes(int64_t B, int64_t T, int64_t K);
// K <= 8, T <= 1024: parallel in time, one wave per 64-step segment (hmm_seg.hip)
bool fwdbwd_seg_ok(int64_t B, int64_t T, int64_t K);
int launch_fwdbwd_seg(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                      int64_t T, int64_t K, float* gamma, float* logZ, float* ws, hipStream_t s);
int launch_viterbi(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                   int64_t T, int64_t K, int32_t* path, float* score, void* ws, size_t ws_bytes, hipStream_t s);
int launch_fwdbwd(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                  int64_t T, int64_t K, float* gamma, float* logZ, void* ws, size_t ws_bytes, hipStream_t s);
int launch_clip_grad_norm(float* g, int64_t n, float pre_scale, float max_norm, float* total_out, hipStream_t s);
int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1, double beta2,
                double eps, int64_t* step, float gmul, hipStream_t s);

}  // namespace vqhmm
