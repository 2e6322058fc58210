/* vqhmm — C-ABI of the MI355X-native VAE_HMM hot path (libvqhmm.so, gfx950).
 *
 * The reference (yashnaray/VQ-VAE-HMM-model) is pure Python/PyTorch and exposes
 * no FFI: its boundary is the nn.Module surface of VQ_VAE_HMM_fixed.py.  Each
 * entry point below replaces the ATen work behind one piece of that surface
 * (citations per function).  The Python package `vqhmm` binds these with
 * ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer (allocated by the caller, e.g. the
 *    PyTorch caching allocator) unless documented otherwise; the library never
 *    allocates, frees or synchronises.  Scratch memory is a caller-provided
 *    workspace whose size comes from the matching *_workspace_size query.
 *  - Work is enqueued on `stream` (a hipStream_t; NULL = default stream) and
 *    is asynchronous; kernel faults surface at the caller's next sync.
 *  - Return value: 0 on success, negative VQHMM_E* code on bad arguments or a
 *    failed launch.  No global mutable state: calls are reentrant from any
 *    host thread with its own stream, and graph-capturable.
 *  - Tensors are dense row-major in the reference's layouts: "CF" = (B, C, T)
 *    channels-first as nn.Conv1d uses; log_A is (B, T, K, K) with index t the
 *    transition t-1 -> t (VQ_VAE_HMM_fixed.py:69,125-127).
 *  - fp32 throughout (the reference computes in fp32).
 */
#ifndef VQHMM_H
#define VQHMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VQHMM_OK 0
#define VQHMM_EINVAL -1
#define VQHMM_ELAUNCH -2
#define VQHMM_EWORKSPACE -3
#define VQHMM_EUNSUPPORTED -4

/* Bits of the training step's device status word (vqhmm_elbo_status_offset).  Kernels only
 * ever OR bits in; the caller zeroes the word when it allocates the workspace and reads it
 * after a synchronisation (TrainState.check_status raises RuntimeError on any bit). */
#define VQHMM_STATUS_TAIL_TIMEOUT 1ull /* reserved: no kernel sets it (no launch waits on another
                                          * workgroup); kept so callers' status checks stay valid */

/* Number of parameter tensors of a VAE_HMM, in nn.Module.parameters() order
 * (VQ_VAE_HMM_fixed.py:92-98 -> encoder :32-36, prior :44-57, decoder :74-79). */
#define VQHMM_NPARAMS 18

/* Constructor arguments of VAE_HMM(input_dim, hidden_dim, K, hidden_dim2,
 * u_dim, trans_hidden)  (VQ_VAE_HMM_fixed.py:93). */
typedef struct vqhmm_dims {
  int32_t input_dim;    /* D  */
  int32_t hidden_dim;   /* H  (encoder conv1, decoder embedding + convs) */
  int32_t K;            /* number of regimes */
  int32_t hidden_dim2;  /* H2 (encoder conv2) */
  int32_t u_dim;        /* U  */
  int32_t trans_hidden; /* TH */
} vqhmm_dims_t;

/* Library ABI version (bumped on any signature change). */
int32_t vqhmm_abi_version(void);

/* Element offsets of the 18 parameters inside one flat fp32 buffer laid out
 * in parameters() order; offsets[18] = total element count.  Host-only. */
int vqhmm_param_layout(const vqhmm_dims_t* dims, int64_t offsets[VQHMM_NPARAMS + 1]);

/* ---------------------------------------------------------------- VQ ----
 * Nearest-codeword quantization (semantics pseudocode.txt:11
 * `quantize`, hard regimes backtesting.py:154-155 — no reference code).
 * z (B, Dv, T) CF, codebook (K, Dv) -> idx (B, T) int32, dmin (B, T) fp32
 * (nullable).  Expansion form ||z||^2 + ||c_k||^2 - 2 z.c_k, evaluated as
 * s_k = fmaf chain over d ascending of z_d * (-2 c_kd) starting from
 * ||c_k||^2 (itself the fmaf chain of c_kd^2); idx = first k with the
 * smallest s_k; dmin = s_idx + ((q0 + q1) + (q2 + q3)), q_r the fmaf chain of
 * z_d^2 over d = r (mod 4).  Bit-exact vs oracle/c/hmm_oracle.c. */
int vqhmm_vq_argmin_f32(const float* z, int64_t B, int64_t Dv, int64_t T,
                        const float* codebook, int64_t K,
                        int32_t* idx, float* dmin, void* stream);


/* VQ-VAE quantizer (pseudocode.txt:12-18: `z_q, idx = quantize(z_e, codebook)`, the
 * straight-through z_e + (z_q - z_e).detach() of :13 and the commit / codebook MSEs of :17-18)
 * on channels-first z (B, Dv, T): idx as vqhmm_vq_argmin_f32 (same bit-exact contract),
 * z_q_st[b][d][t] = z + (c[idx][d] - z) in fp32 (the forward value of the straight-through
 * tensor), and *sse = sum over (b, d, t) of (z - c[idx][d])^2 in the direct-difference form,
 * accumulated in fp64 (commit = beta * sse / (B Dv T), codebook loss = sse / (B Dv T)).  Fused in
 * the argmin kernel's epilogue where its row-load path runs (Dv in {4,8,16,32,64}, T % 4 == 0,
 * K <= 32), else argmin + one gather launch; then one fixed-order partial-sum launch (the result
 * is deterministic).  Replaces the reference's `quantize` + two MSEs.
 * Workspace: vqhmm_vq_quantize_workspace_size(B, Dv, T, K) bytes. */
size_t vqhmm_vq_quantize_workspace_size(int64_t B, int64_t Dv, int64_t T, int64_t K);
int vqhmm_vq_quantize_f32(const float* z, int64_t B, int64_t Dv, int64_t T, const float* codebook, int64_t K,
                          int32_t* idx, float* z_q_st, double* sse, void* workspace, size_t ws_bytes,
                          void* stream);

/* ------------------------------------------------------------ Viterbi ----
 * MAP state path (semantics math.md:23-67 over Prior.forward's
 * tables VQ_VAE_HMM_fixed.py:59-71 — no reference code).  log_pi (K),
 * log_A (B,T,K,K) [t = transition t-1 -> t], em (B,T,K) emission log-potentials,
 * lengths (B) int64 -> path (B,T) int32 (-1 at t >= length), score (B) fp32.
 * d_t[j] = (max_i d_{t-1}[i] + log_A[t,i,j]) + em[t,j] in fp32, ties -> lowest i;
 * last state = first argmax.  Bit-exact vs oracle/c/hmm_oracle.c.  K <= 4096 (K <= 8: packed lane
 * groups, hmm.hip; 8 < K <= 32: one sequence per wave, hmm_wide.hip; 32 < K <= 4096: one workgroup
 * per sequence, states j, j + 256, .. per thread, 16-bit backpointers past 256 states,
 * hmm_generic.hip); larger K -> VQHMM_EUNSUPPORTED.
 * Workspace: vqhmm_viterbi_workspace_size(B, T, K) bytes (backpointers as one
 * 64-bit lane ballot per step per wave of 64 / KP^2 sequences, KP = K rounded
 * up to a power of two; T rounded up to 64). */
size_t vqhmm_viterbi_workspace_size(int64_t B, int64_t T, int64_t K);
int vqhmm_viterbi_f32(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                      int64_t B, int64_t T, int64_t K, int32_t* path, float* score, void* workspace,
                      size_t ws_bytes, void* stream);

/* --------------------------------------------------- forward-backward ----
 * Posterior marginals: same inputs as Viterbi ->
 * gamma (B,T,K) fp32 (0 at t >= length), logZ (B) fp32 (NaN if length 0).
 * Base-2 log-space alpha/beta with per-step shifts; a chunk whose fast step
 * leaves float range is recomputed with the max-shifted log-sum-exp.  For
 * 2 <= K <= 8 and 128 <= T <= 1024 (K = 4: T > 256) the kernel is parallel in
 * time (64-step segments' transfer matrices on the matrix cores, a boundary
 * pass, then per-segment chains; hmm_seg.hip); a sequence that leaves the
 * linear range there is recomputed exactly in the same launch.
 * Workspace: vqhmm_fwdbwd_workspace_size(B, T, K) = 2 * B * T * K * 4 bytes.
 * Accuracy target vs the fp64 oracle: |gamma| abs 1e-5, logZ rel 1e-5.  K <= 4096 (as Viterbi). */
size_t vqhmm_fwdbwd_workspace_size(int64_t B, int64_t T, int64_t K);
int vqhmm_fwdbwd_f32(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths,
                     int64_t B, int64_t T, int64_t K, float* gamma, float* logZ, void* workspace,
                     size_t ws_bytes, void* stream);

/* ------------------------------------------------------- training step ----
 * compute_loss forward + backward of VAE_HMM (VQ_VAE_HMM_fixed.py:106-137,
 * autograd of :156) as one native executor over hand-written kernels.
 *
 * params: host array of VQHMM_NPARAMS device pointers in parameters() order
 *   (shapes: the reference's nn.Conv1d / nn.Linear / nn.Embedding weights).
 * x (B, D, T) CF; u (B, U, T) if u_layout == 0, (B, T, U) if u_layout == 1
 *   (Prior.forward's permute rule, :64-65); lengths (B) int64 on device.
 * Workspace: vqhmm_elbo_workspace_size(); the forward saves activations in it
 * and the backward must get the same workspace, dims, B and T.
 * loss: device fp32 scalar; loss_accum (nullable): device fp64 scalar += loss
 *   (train_model's epoch_loss, :158, without a per-step host sync).
 * need_grad = 0 computes only the loss; 2 = as 1, but the loss (and loss_accum) are left to the
 *   backward: vqhmm_elbo_bwd_adam_f32 or vqhmm_elbo_bwd_loss_f32 with its loss pointers finalizes
 *   them in its own last launch (one launch fewer per step).
 * norm: NULL, or a device int64[2] {valid_count, batch} replacing the batch's own
 *   loss normalisers mask.sum() (:120) and B (:131, :135).  Pass the GLOBAL batch's
 *   values when this batch is one shard of it: the shards' losses and gradients then
 *   SUM to the global batch's exactly (data parallel over ragged batches).  The
 *   backward must get the same norm as its forward.
 * Backward: grad (flat fp32, vqhmm_param_layout order) = grad_scale * dloss/dparams,
 *   grad_scale a device fp32 scalar (autograd's grad_output) or NULL for 1. */
int vqhmm_elbo_workspace_size(const vqhmm_dims_t* dims, int64_t B, int64_t T, size_t* bytes);
int vqhmm_elbo_fwd_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                       const float* u, int u_layout, const int64_t* lengths, const int64_t* norm, int64_t B, int64_t T,
                       float beta, int need_grad, void* workspace, size_t ws_bytes,
                       float* loss, double* loss_accum, void* stream);
int vqhmm_elbo_bwd_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                       const int64_t* norm, int64_t B, int64_t T, float beta, const float* grad_scale,
                       void* workspace, size_t ws_bytes, float* grad, void* stream);
/* vqhmm_elbo_bwd_f32 that also finalizes the loss of a forward run with need_grad = 2 into loss /
 * loss_accum (the data-parallel step form: forward + backward, then the gradient all-reduce and
 * vqhmm_adam_f32; VQ_VAE_HMM_fixed.py:137,156,158). */
int vqhmm_elbo_bwd_loss_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                            const int64_t* norm, int64_t B, int64_t T, float beta, const float* grad_scale,
                            void* workspace, size_t ws_bytes, float* grad, float* loss, double* loss_accum,
                            void* stream);
/* Backward + torch.optim.Adam step (the single-process train_model step,
 * VQ_VAE_HMM_fixed.py:155-157): vqhmm_elbo_bwd_f32 (grad_scale NULL) whose last launch
 * also applies vqhmm_adam_f32's update to every parameter element (same formula, same
 * device step counter and ticket), saving the separate update launch; grad still receives
 * the full gradient.  params[i] must be param + offset[i] of vqhmm_param_layout (the flat
 * buffer Adam updates in place).  adam_grad_scale multiplies the gradient inside Adam only.
 * loss / loss_accum: NULL, or (after a forward with need_grad = 2) where the forward's loss is
 * finalized, as vqhmm_elbo_fwd_f32 would have. */
int vqhmm_elbo_bwd_adam_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                            const int64_t* norm, int64_t B, int64_t T, float beta, void* workspace,
                            size_t ws_bytes, float* grad, float* param, float* exp_avg, float* exp_avg_sq,
                            double lr, double beta1, double beta2, double eps, int64_t* step,
                            float adam_grad_scale, float* loss, double* loss_accum, void* stream);
/* Device addresses (inside the workspace) of the last forward's loss and of its
 * pieces [recon, prior, entropy] (for tests).  Host-only, no GPU access. */
int vqhmm_elbo_pieces(const vqhmm_dims_t* dims, int64_t B, int64_t T, const void* workspace,
                      const float** loss, const float** pieces);

/* Byte offset, inside an elbo workspace of this (dims, B, T), of the step's 8-byte device
 * status word (VQHMM_STATUS_* bits).  The caller zeroes it once after allocating the
 * workspace; the step's kernels never clear it.  Host-only. */
int vqhmm_elbo_status_offset(const vqhmm_dims_t* dims, int64_t B, int64_t T, size_t* offset);

/* Device addresses (inside the workspace) of the step's PCL activation and gradient
 * buffers, in this order: x, h1, h2, logits, q, g1, g2, par (mu|logvar), dpar, dg2, dg1,
 * dq(decoder), dlogits, dh2, dh1, dq(prior).  Row r = b*(T+2)+1+t, stride ld4(channels).
 * Host-only, for accuracy diagnostics (tools/grad_accuracy.py). */
int vqhmm_elbo_debug_buffers(const vqhmm_dims_t* dims, int64_t B, int64_t T, const void* workspace,
                             const float** buffers16);

/* Phase timestamps (s_memrealtime ticks, 100 MHz) of the last launch of a kernel family built for
 * profiling (which = 0: the strip kernels, VQHMM_STRIP_PROF=1; 1: the conv2 kernels, VQHMM_CONV_PROF=1;
 * 2: the cooperative ELBO head, VQHMM_HEAD_PROF=1;
 * the switches are read once; results unchanged): 16 slots per workgroup for the first 256
 * workgroups.  Host-only, synchronous (tools/strip_prof.py). */
int vqhmm_debug_prof(int which, uint64_t* out, int64_t n);

/* Stage table of the training step (forward stages then backward stages, in
 * launch order).  stage_info: name, algorithmic FLOPs and bytes of ONE launch
 * (host-only); stage_f32 re-runs one stage on a workspace holding a completed
 * forward/backward (per-kernel timing, ablation). */
int vqhmm_elbo_num_stages(void);
int vqhmm_elbo_stage_info(const vqhmm_dims_t* dims, int64_t B, int64_t T, int stage, char* name,
                          size_t name_len, double* flops, double* bytes, int* mfma_bound);
int vqhmm_elbo_stage_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                         const float* u, int u_layout, const int64_t* lengths, const int64_t* norm,
                         int64_t B, int64_t T, float beta, void* workspace, size_t ws_bytes, float* grad, int stage,
                         void* stream);

/* torch.optim.Adam step (no weight decay / amsgrad; train_model uses the
 * defaults, :146) over n contiguous fp32 elements.  `step` is a DEVICE int64
 * step counter that this call increments before the update (so a captured
 * graph replays correct bias corrections).  The update and the increment are
 * one launch: during it the upper 32 bits hold a completion ticket, so between
 * calls *step is the plain step count and must stay below 2^32.  The gradient is multiplied by
 * grad_scale first (1/world_size after a SUM all-reduce, else 1). */
int vqhmm_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   double lr, double beta1, double beta2, double eps, int64_t* step, float grad_scale,
                   void* stream);

/* torch.nn.utils.clip_grad_norm_(parameters, max_norm) over the flat gradient
 * (Trainer.train_epoch, src/training/trainer.py:32): grad *= pre_scale, then
 * total = ||grad||_2 and grad *= min(max_norm / (total + 1e-6), 1), all on the
 * device.  total_norm (nullable, device fp32) receives the norm, which is what
 * clip_grad_norm_ returns.  pre_scale folds the 1/world of a SUM all-reduce in
 * before the norm.  Follow with vqhmm_adam_f32(..., grad_scale = 1). */
int vqhmm_clip_grad_norm_f32(float* grad, int64_t n, float pre_scale, float max_norm, float* total_norm,
                             void* stream);

/* ---------------------------------------------------------- data step ----
 * RandomChunkDataset.__getitem__ (:25-29) + collate_fn (:164-179) on the
 * device: out (B, C, Tmax) = zero-padded chunks, out[i,c,t] = t < L_i ?
 * src[base_i + c*n_i + s_i + t] : 0, with meta (B x 4 int64, device) =
 * {base_i, n_i, s_i, L_i} per sample (a row-major (C, n_i) sequence at element
 * base_i of src, chunk start s_i, length L_i).  Bit-identical to collate_fn. */
int vqhmm_gather_chunks_f32(const float* src, const int64_t* meta, int64_t B, int64_t C, int64_t Tmax,
                            float* out, void* stream);

/* ---------------------------------------------------------- inference ----
 * VAE_HMM.encode (:100, Encoder.forward :38-41): x (B,D,T) -> logits (B,K,T)
 * VAE_HMM.decode (:103, Decoder.forward :81-90): q (B,K,T) -> mu, logvar (B,D,T)
 * VAE_HMM.forward (:139-143): x -> mu, logvar, q = softmax(logits, dim=1)
 * Prior.forward (:59-71): u -> log_pi (K), log_A (B,T,K,K)
 * Unused parameter pointers may be NULL (e.g. encode needs only the encoder's). */
int vqhmm_infer_workspace_size(const vqhmm_dims_t* dims, int64_t B, int64_t T, size_t* bytes);
int vqhmm_encode_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                     int64_t B, int64_t T, float* logits, void* workspace, size_t ws_bytes, void* stream);
int vqhmm_decode_f32(const vqhmm_dims_t* dims, const float* const* params, const float* q,
                     int64_t B, int64_t T, float* mu, float* logvar, void* workspace, size_t ws_bytes,
                     void* stream);
int vqhmm_forward_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                      int64_t B, int64_t T, float* mu, float* logvar, float* q, void* workspace,
                      size_t ws_bytes, void* stream);
int vqhmm_prior_f32(const vqhmm_dims_t* dims, const float* const* params, const float* u, int u_layout,
                    int64_t B, int64_t T, float* log_pi, float* log_A, void* stream);
/* Autograd of the module surface (VAE_HMM.encode / decode / forward under torch autograd, :100-104,
 * :139-143; examples/backtest_example.py:30 calls encode with grad enabled).  Each recomputes its module's
 * forward into the workspace (vqhmm_module_bwd_workspace_size), then runs the data gradients, the weight
 * gradients and one fixed-order slab reduction.  grad: the flat buffer of vqhmm_param_layout(dims); only the
 * module's own entries are written (encode: encoder.*; decode: decoder.*; forward: both).  Output gradients
 * are channels-first like the outputs: dlogits (B,K,T); dpar = [dmu | dlogvar] (B,2D,T); dq (B,K,T) the
 * gradient of forward's q output (NULL: 0; forward's dpar NULL: 0).  Input gradients dx (B,D,T) / dq (B,K,T)
 * are written when non-NULL. */
int vqhmm_module_bwd_workspace_size(const vqhmm_dims_t* dims, int64_t B, int64_t T, size_t* bytes);
int vqhmm_encode_bwd_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                         const float* dlogits, int64_t B, int64_t T, void* workspace, size_t ws_bytes,
                         float* grad, float* dx, void* stream);
int vqhmm_decode_bwd_f32(const vqhmm_dims_t* dims, const float* const* params, const float* q,
                         const float* dpar, int64_t B, int64_t T, void* workspace, size_t ws_bytes,
                         float* grad, float* dq, void* stream);
int vqhmm_forward_bwd_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x,
                          const float* dpar, const float* dq, int64_t B, int64_t T, void* workspace,
                          size_t ws_bytes, float* grad, float* dx, void* stream);
/* Autograd of Prior.forward (VQ_VAE_HMM_fixed.py:59-71) alone: dlog_pi (K, nullable = 0) and dlog_A
 * (B,T,K,K) -> grad's prior.* entries (log_prior, transition_net.0/.2 weight and bias; nothing else is
 * written) and du (nullable; CF (B, U, T) whatever u_layout).  Recomputes the MLP into the workspace
 * (vqhmm_prior_bwd_workspace_size), then the log_softmax backwards, the hidden layer's masked data
 * gradient, du, the two weight gradients and one fixed-order slab reduction. */
int vqhmm_prior_bwd_workspace_size(const vqhmm_dims_t* dims, int64_t B, int64_t T, size_t* bytes);
int vqhmm_prior_bwd_f32(const vqhmm_dims_t* dims, const float* const* params, const float* u, int u_layout,
                        const float* dlog_pi, const float* dlog_A, int64_t B, int64_t T, void* workspace,
                        size_t ws_bytes, float* grad, float* du, void* stream);

/* ------------------------------------------- fused Prior -> Viterbi ----
 * the Viterbi path of vqhmm_viterbi_f32 over the tables vqhmm_prior_f32 would write
 * (Prior.forward VQ_VAE_HMM_fixed.py:59-71), computed per chunk on the chip from u and never stored:
 * HBM reads u (4U B per position) instead of log_A (4K^2 B, written then read).  u as in
 * vqhmm_prior_f32 (u_layout 0: (B,U,T), 1: (B,T,U)); em (B,T,K); lengths (B) int64 ->
 * path (B,T) int32, score (B).  path / score equal vqhmm_viterbi_f32 on vqhmm_prior_f32's log_pi and
 * log_A bit for bit.  K <= 8, u_dim <= 4, trans_hidden in {64, 128, 256}; other dims ->
 * VQHMM_EUNSUPPORTED (run vqhmm_prior_f32 + vqhmm_viterbi_f32).  Workspace:
 * vqhmm_prior_viterbi_workspace_size(dims, B, T) bytes. */
size_t vqhmm_prior_viterbi_workspace_size(const vqhmm_dims_t* dims, int64_t B, int64_t T);
int vqhmm_prior_viterbi_f32(const vqhmm_dims_t* dims, const float* const* params, const float* u, int u_layout,
                            const float* em, const int64_t* lengths, int64_t B, int64_t T, int32_t* path,
                            float* score, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------- hard regimes ----
 * regime_probs.argmax(dim=1) of softmax(encode(x), dim=1) — backtesting.py:154-155,
 * src/backtesting.py:105-107, VQ_VAE+HMM.ipynb:830, visualize.ipynb:74.  One fused
 * pass: the encoder's to_logits epilogue computes q and its first argmax.
 * x (B,D,T) -> regimes (B,T) int32 and, if q != NULL, q (B,K,T) fp32 (the probabilities
 * the argmax was taken over).  Argmax rule = torch.argmax: NaN is the maximum, the
 * lowest index wins ties; so regimes == q.argmax(dim=1) bit for bit.  Workspace:
 * vqhmm_infer_workspace_size. */
int vqhmm_regimes_f32(const vqhmm_dims_t* dims, const float* const* params, const float* x, int64_t B, int64_t T,
                      float* q, int32_t* regimes, void* workspace, size_t ws_bytes, void* stream);
/* Same argmax rule over the channel axis of any CF tensor: q (B,K,T) -> idx (B,T) int32. */
int vqhmm_argmax_f32(const float* q, int64_t B, int64_t K, int64_t T, int32_t* idx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VQHMM_H */
