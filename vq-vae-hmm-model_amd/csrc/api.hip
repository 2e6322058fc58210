// extern "C" entry points of libvqhmm.so (declared in include/vqhmm.h) and the
// native executor of the VAE_HMM training step: it plans the workspace and
// enqueues the forward (5 kernels + finalize) and backward (~16 kernels)
// passes on the caller's stream.  See DESIGN.md for the kernel list.
#include "vqhmm.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "kernels.h"


using namespace vqhmm;

namespace {

enum P {
  ENC1_W, ENC1_B, ENC2_W, ENC2_B, LOGIT_W, LOGIT_B, LOG_PRIOR, TN0_W, TN0_B, TN2_W, TN2_B,
  EMB, DEC1_W, DEC1_B, DEC2_W, DEC2_B, PAR_W, PAR_B
};

struct Carver {
  char* base;
  size_t off = 0;
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

// Head choice (VQHMM_HEAD, read once): default the workgroup-cooperative head (head_coop.hip) wherever it
// applies, pipelined (one 12-wave workgroup per CU, elbo_head_pipe_kernel) for K <= 4, TH = 128; "coop" = the
// two-workgroups-per-CU form for K <= 4 too, "tile" = the tile-barrier MFMA head (head_mfma.hip) — A/B
// switches.
int head_choice() {
  static const int v = [] {
    const char* e = VQHMM_ENV("VQHMM_HEAD");
    if (e && strcmp(e, "tile") == 0) return 2;
    if (e && strcmp(e, "coop") == 0) return 3;
    return 0;
  }();
  return v;
}

// A/B switches, read once: VQHMM_WGROUP=0 launches the six weight gradients separately;
// VQHMM_WGRAD_MINROWS = the grouped launch's minimum rows per chunk (multiple of 64).
bool wgroup_enabled() {
  static const bool v = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGROUP");
    return !(e && e[0] == '0');
  }();
  return v;
}
// Grouped weight gradients: dec_conv2's 64 x 64 x 3 job as two 32-output halves (VQHMM_WGRAD_SPLIT, read
// once): twice the workgroups, each half-length, on the enc_conv2 body.
bool wgrad_split_on() {
  static const bool v = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_SPLIT");
    return e && e[0] == '1';
  }();
  return v;
}
int64_t wgroup_min_rows() {
  static const int64_t v = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_MINROWS");
    // 3 stages: fewer, fuller slabs at small batches (B = 128: 64 / 128 / 192 / 256 rows 0.1463 / 0.1381 /
    // 0.1369 / 0.1377 ms; B = 256: 128 -> 192 rows 0.1953 -> 0.1921 ms)
    const long r = e ? atol(e) : 192;
    return (int64_t)(r >= 64 && r <= 65536 && r % 64 == 0 ? r : 192);
  }();
  return v;
}

// VQHMM_STRIP=0: the forward convolutions as pair launches; VQHMM_STRIP_HEAD=1: the ELBO head fused into the
// forward strip (A/B switches, read once).  The fused head is off by default: one 8-wave workgroup per CU runs
// the head's phases in lockstep behind its barriers, where head_coop's two workgroups per CU overlap one's
// VALU phase with the other's MFMA phase, so it measured slower (strip + head: B = 128 46.6 -> 43.2 us but the
// step 0.1161 -> 0.1162 ms; cfg2 178 -> 199 us, 0.462 -> 0.488 ms; gpurun_out sq7)
bool strip_fwd_env() {
  static const bool on = [] {
    const char* e = VQHMM_ENV("VQHMM_STRIP");
    return !e || atoi(e) != 0;
  }();
  return on;
}
bool strip_head_on() {
  static const bool on = [] {
    const char* e = VQHMM_ENV("VQHMM_STRIP_HEAD");
    return e && atoi(e) != 0;
  }();
  return on && strip_fwd_env();
}
// VQHMM_STRIP_WGRAD=0: the backward strip without the weight gradients (they then run as the grouped
// wgrad2 launch), A/B switch read once.  The fold sums each weight gradient in another order (per strip
// workgroup instead of per row chunk), so the two forms agree within rounding, not bit for bit
bool strip_wgrad_env() {
  static const bool on = [] {
    const char* e = VQHMM_ENV("VQHMM_STRIP_WGRAD");
    return !e || atoi(e) != 0;
  }();
  return on;
}
// the shapes the forward strip covers (strip_fwd_supported on the plan's ConvArgs agrees)
bool strip_fwd_shapes_ok(int D, int H, int H2, int K, int64_t R) {
  return D >= 1 && 3 * D <= 16 && H == 64 && H2 >= 1 && H2 <= 32 && K >= 1 && K <= 4 && R > 0 && R < (1ll << 31);
}

bool dims_ok(const vqhmm_dims_t* d) {
  return d && d->input_dim > 0 && d->hidden_dim > 0 && d->K > 0 && d->hidden_dim2 > 0 && d->u_dim > 0 &&
         d->trans_hidden > 0;
}

// Wgrad problem descriptors of the 6 convolutions, in backward order.
struct WLayer {
  int N, C, ks;
  int64_t rows, nchunks;
  float* slab;
  float* bslab;
  float* cslab;  // the composed decoder conv1 (wl[2], grouped launch): per-chunk dE shares [nchunks][K][H]
};

struct ElboPlan {
  int64_t B, R;
  int T, D, H, H2, K, U, TH;
  int hgrid;
  // forward (PCL buffers, row stride ld4(channels))
  float *xp, *up;
  float *h1e, *h2e, *logits, *q, *g1, *g2, *par, *Wc;
  // head
  float *dpar, *dqx, *dlx;
  double* part;
  float *sW1, *sb1, *sW2, *sb2, *sq0;
  float *loss, *pieces;
  int64_t* cnt;  // valid count written by the prologue (loss finalized in the backward)
  unsigned long long* sync;  // [2] the status word (vqhmm_elbo_status_offset; reserved), [0], [1], [3] spare
  // staged head (shapes the fused heads do not cover): Prior MLP as 1x1 convs
  bool staged;
  bool coop_head;  // head_coop.hip (K <= 8, the default); else head_mfma / head.hip
  bool pipe_head;  // ... its pipelined kernel (K <= 4)
  bool dec2_split; // grouped weight gradients: dec_conv2's job as two 32-output halves (slabs [half][chunk][32]..)
  bool strip_head;  // the head runs inside the forward strip launch (strip.hip; slabs = its workgroups)
  float *hid, *lgA, *dhid, *nx, *dqc, *trw, *logpi;
  // backward
  float *dg2, *dg1, *dqd, *dlog, *dh2, *dh1, *dWc;
  float *Ecopy, *Wcopy;  // the prologue's copies of decoder.embeddings / decoder.conv1 weights, read by the
                         // launch that also Adam-updates them (tail: E; compose_adam: both; Wcopy null when grouped)
  float* himg;           // the cooperative head's weight image (built by the prologue), or null
  bool wgroup;           // the six weight gradients run as one grouped launch (wgrad2_group)
  bool wfold;            // ... or inside the backward strip launch (strip_bwdw.hip; slabs = its workgroups).
                         // Either way the tail sees the grouped layout (composed segment + dE shares)
  int nwl;
  WLayer wl[8];  // 0 to_params, 1 dec2, 2 dec1', 3 to_logits, 4 enc2, 5 enc1, [6 Prior W1, 7 Prior W2]
  float* img[32];  // per stage: packed conv2_kernel weight image (WImgJob), built by the prologue, or null
  size_t bytes;
};

void plan_images(ElboPlan& p, Carver& c);
bool strip_wfold_planned(const ElboPlan& p);

ElboPlan plan_elbo(const vqhmm_dims_t* d, int64_t B, int64_t T, void* ws) {
  // size / shape queries: carve from a non-null base (kernel choices test pointers for presence;
  // nothing is dereferenced), so the plan is exactly the one a real workspace gets
  if (!ws) return plan_elbo(d, B, T, reinterpret_cast<void*>(4096));
  ElboPlan p{};
  p.B = B; p.T = (int)T; p.R = B * (T + 2);
  p.D = d->input_dim; p.H = d->hidden_dim; p.H2 = d->hidden_dim2; p.K = d->K; p.U = d->u_dim; p.TH = d->trans_hidden;
  const int64_t R = p.R;
  const int H = p.H, H2 = p.H2, K = p.K, D = p.D;
  Carver c{reinterpret_cast<char*>(ws)};
  p.xp = c.take<float>(R * ld4(D));
  p.up = c.take<float>(R * ld4(p.U));
  p.h1e = c.take<float>(R * ld4(H));
  p.h2e = c.take<float>(R * ld4(H2));
  p.logits = c.take<float>(R * ld4(K));
  p.q = c.take<float>(R * ld4(K));
  p.g1 = c.take<float>(R * ld4(H));
  p.g2 = c.take<float>(R * ld4(H));
  p.par = c.take<float>(R * ld4(2 * D));
  p.Wc = c.take<float>((size_t)H * K * 3);
  {
    HeadArgs hc{};
    hc.K = K; hc.U = p.U; hc.TH = p.TH; hc.D = D;
    hc.R = R;
    p.coop_head = head_coop_supported(hc) && (head_choice() == 0 || head_choice() == 3);
    p.pipe_head = p.coop_head && head_pipe_supported(hc) && head_choice() == 0;
  }
  {
    HeadArgs hc{};
    hc.K = K; hc.U = p.U; hc.TH = p.TH; hc.D = D; hc.R = R;
    p.strip_head = p.coop_head && strip_head_on() && strip_fwd_shapes_ok(D, H, H2, K, R) && strip_head_supported(hc);
  }
  p.hgrid = p.strip_head ? strip_fwd_grid(R)
            : p.pipe_head ? head_pipe_grid(R) : p.coop_head ? head_coop_grid(R, K) : head_grid(R);
  p.dpar = c.take<float>(R * ld4(2 * D));
  p.dqx = c.take<float>(R * ld4(K));
  p.dlx = c.take<float>(R * ld4(K));
  p.part = c.take<double>((size_t)p.hgrid * 4);
  {
    HeadArgs hc{};
    hc.K = K; hc.U = p.U; hc.TH = p.TH; hc.D = D;
    p.staged = !fused_head_supported(hc);
  }
  if (!p.staged) {
    p.sW1 = c.take<float>((size_t)p.hgrid * p.TH * p.U);
    p.sb1 = c.take<float>((size_t)p.hgrid * p.TH);
    p.sW2 = c.take<float>((size_t)p.hgrid * K * K * p.TH);
    p.sb2 = c.take<float>((size_t)p.hgrid * K * K);
    p.sq0 = c.take<float>((size_t)p.hgrid * K);
  } else {
    p.sq0 = c.take<float>(K);  // one chunk: q summed over the t = 0 rows
    p.hid = c.take<float>(R * ld4(p.TH));
    p.lgA = c.take<float>(R * ld4(K * K));
    p.dhid = c.take<float>(R * ld4(p.TH));
    p.nx = c.take<float>(R * ld4(K));
    p.dqc = c.take<float>(R * ld4(K));
    p.trw = c.take<float>(R);
    p.logpi = c.take<float>(K);
  }
  p.loss = c.take<float>(1);
  p.pieces = c.take<float>(4);
  p.cnt = c.take<int64_t>(1);
  p.sync = c.take<unsigned long long>(4);
  p.dg2 = c.take<float>(R * ld4(H));
  p.dg1 = c.take<float>(R * ld4(H));
  p.dqd = c.take<float>(R * ld4(K));
  p.dlog = c.take<float>(R * ld4(K));
  p.dh2 = c.take<float>(R * ld4(H2));
  p.dh1 = c.take<float>(R * ld4(H));
  p.dWc = c.take<float>((size_t)H * K * 3);
  p.himg = p.coop_head ? c.take<float>((size_t)head_coop_image_floats(K, p.TH)) : nullptr;
  p.Ecopy = c.take<float>((size_t)K * H);
  const int shapes[8][3] = {{2 * D, H, 1}, {H, H, 3}, {H, K, 3}, {K, H2, 1}, {H2, H, 3}, {H, D, 3},
                            {p.TH, p.U, 1}, {K * K, p.TH, 1}};
  p.nwl = p.staged ? 8 : 6;
  p.wgroup = wgroup_enabled();
  for (int i = 0; i < 6; ++i) {
    WgradArgs t{};
    t.N = shapes[i][0]; t.C = shapes[i][1]; t.ks = shapes[i][2];
    if (i == 2) t.cmpW = reinterpret_cast<const float*>(4096);  // the composed layer's dE epilogue (shape check only)
    p.wgroup = p.wgroup && wgrad2_group_supported(t);
  }
  // the grouped path's tail forms the composed dW itself (a block reduces <= 256 dWc columns)
  p.wgroup = p.wgroup && composed_block_cols(H, K) <= 256;
  p.Wcopy = p.wgroup ? nullptr : c.take<float>((size_t)H * H * 3);
  plan_images(p, c);
  p.wfold = p.wgroup && strip_wfold_planned(p);
  p.dec2_split = p.wgroup && !p.wfold && wgrad_split_on() && H == 64;
  for (int i = 0; i < p.nwl; ++i) {
    WLayer& w = p.wl[i];
    w.N = shapes[i][0]; w.C = shapes[i][1]; w.ks = shapes[i][2];
    const int64_t tiles = cdiv(w.N, 64) * cdiv(w.C, 64);
    WgradArgs probe{};
    probe.N = w.N; probe.C = w.C; probe.ks = w.ks; probe.rows_per_chunk = 64;
    w.rows = (w.N <= 64 && w.C <= 64) ? wgrad2_rows(R, w.N, w.C, w.ks)
             : wgradbig_supported(probe) ? wgradbig_rows(R, w.N, w.C) : wgrad_chunks(R, tiles);
    if (i < 6 && p.wgroup) w.rows = wgrad2_group_rows(std::max<int64_t>(w.rows, wgroup_min_rows()), w.N, w.C, w.ks);
    if (i < 6 && p.wfold) w.rows = cdiv(R, strip_bwdw_grid(R));  // one slab row per strip workgroup
    w.nchunks = (i < 6 && p.wfold) ? strip_bwdw_grid(R) : cdiv(R, w.rows);
    w.slab = c.take<float>((size_t)w.nchunks * w.N * w.C * w.ks);
    w.bslab = c.take<float>((size_t)w.nchunks * w.N);
    w.cslab = (i == 2 && p.wgroup) ? c.take<float>((size_t)w.nchunks * K * H) : nullptr;
  }
  p.bytes = c.off + 256;
  return p;
}

ConvArgs conv_base(const ElboPlan& p) {
  ConvArgs a{};
  a.R = p.R; a.T = p.T;
  return a;
}

}  // namespace

extern "C" {

int32_t vqhmm_abi_version(void) { return 6; }

int vqhmm_param_layout(const vqhmm_dims_t* d, int64_t off[VQHMM_NPARAMS + 1]) {
  if (!dims_ok(d) || !off) return VQHMM_EINVAL;
  const int64_t D = d->input_dim, H = d->hidden_dim, K = d->K, H2 = d->hidden_dim2, U = d->u_dim,
                TH = d->trans_hidden;
  const int64_t sz[VQHMM_NPARAMS] = {
      H * D * 3, H,        // encoder.conv1
      H2 * H * 3, H2,      // encoder.conv2
      K * H2, K,           // encoder.to_logits
      K,                   // prior.log_prior
      TH * U, TH,          // prior.transition_net.0
      K * K * TH, K * K,   // prior.transition_net.2
      K * H,               // decoder.embeddings
      H * H * 3, H,        // decoder.conv1
      H * H * 3, H,        // decoder.conv2
      2 * D * H, 2 * D,    // decoder.to_params
  };
  off[0] = 0;
  for (int i = 0; i < VQHMM_NPARAMS; ++i) off[i + 1] = off[i] + sz[i];
  return VQHMM_OK;
}

int vqhmm_vq_argmin_f32(const float* z, int64_t B, int64_t Dv, int64_t T, const float* codebook, int64_t K,
                        int32_t* idx, float* dmin, void* stream) {
  if (B < 0 || T < 0 || (B * T > 0 && (!z || !codebook || !idx))) return VQHMM_EINVAL;
  return launch_vq_argmin(z, B, Dv, T, codebook, K, idx, dmin, (hipStream_t)stream);
}

size_t vqhmm_vq_quantize_workspace_size(int64_t B, int64_t Dv, int64_t T, int64_t K) {
  return (B < 0 || T < 0 || Dv < 1 || K < 1) ? 0 : vq_quantize_ws_bytes(B, Dv, T, K);
}

int vqhmm_vq_quantize_f32(const float* z, int64_t B, int64_t Dv, int64_t T, const float* codebook, int64_t K,
                          int32_t* idx, float* z_q_st, double* sse, void* ws, size_t ws_bytes, void* stream) {
  if (B < 0 || T < 0 || Dv < 1 || K < 1 || !sse || !ws || (B * T > 0 && (!z || !codebook || !idx || !z_q_st)))
    return VQHMM_EINVAL;
  return launch_vq_quantize(z, B, Dv, T, codebook, K, idx, z_q_st, sse, ws, ws_bytes, (hipStream_t)stream);
}

size_t vqhmm_viterbi_workspace_size(int64_t B, int64_t T, int64_t K) {
  return (B < 0 || T < 0 || K < 1) ? 0 : viterbi_ws_bytes(B, T, K);
}

int vqhmm_viterbi_f32(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                      int64_t T, int64_t K, int32_t* path, float* score, void* ws, size_t ws_bytes, void* stream) {
  if (B < 0 || T < 0 || K < 1 || (B > 0 && (!log_pi || !log_A || !em || !lengths || !path || !score)))
    return VQHMM_EINVAL;
  if (B == 0 || T == 0) return VQHMM_OK;
  return launch_viterbi(log_pi, log_A, em, lengths, B, T, K, path, score, ws, ws_bytes, (hipStream_t)stream);
}

size_t vqhmm_fwdbwd_workspace_size(int64_t B, int64_t T, int64_t K) {
  return (B < 0 || T < 0 || K < 1) ? 0 : fwdbwd_ws_bytes(B, T, K);
}

int vqhmm_fwdbwd_f32(const float* log_pi, const float* log_A, const float* em, const int64_t* lengths, int64_t B,
                     int64_t T, int64_t K, float* gamma, float* logZ, void* ws, size_t ws_bytes, void* stream) {
  if (B < 0 || T < 0 || K < 1 || (B > 0 && (!log_pi || !log_A || !em || !lengths || !gamma || !logZ)))
    return VQHMM_EINVAL;
  if (B == 0 || T == 0) return VQHMM_OK;
  if (!ws) return VQHMM_EWORKSPACE;
  return launch_fwdbwd(log_pi, log_A, em, lengths, B, T, K, gamma, logZ, ws, ws_bytes, (hipStream_t)stream);
}

int vqhmm_elbo_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* bytes) {
  if (!dims_ok(d) || B < 0 || T < 0 || !bytes) return VQHMM_EINVAL;
  *bytes = plan_elbo(d, B, T, nullptr).bytes;
  return VQHMM_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ stage table
// The training step as an ordered list of kernel launches.  The forward and
// backward entry points run their stages in order; vqhmm_elbo_stage_f32 runs
// one (per-kernel timing / ablation), and vqhmm_elbo_stage_info describes it.
namespace {

enum Stage {
  S_TOPCL, S_COMPOSE, S_ENC1, S_ENC2, S_DEC1, S_DEC2, S_HEAD, S_FINAL,                 // forward
  S_PAR_DG, S_DEC2_DG, S_DEC1_DG, S_LOGIT_BWD, S_LOGIT_DG, S_ENC2_DG,         // backward data
  S_W_PAR, S_W_DEC2, S_W_DEC1, S_W_LOGIT, S_W_ENC2, S_W_ENC1,                 // backward weights
  S_REDUCE, S_COMPOSE_BWD, S_LOGPRIOR,                                         // reductions
  S_COUNT
};
const int FWD_FIRST = S_TOPCL, FWD_LAST = S_FINAL, BWD_FIRST = S_PAR_DG, BWD_LAST = S_LOGPRIOR;
const char* kStageNames[S_COUNT] = {
    "inputs_to_pcl+compose_fwd", "(compose_fwd: in prologue)", "enc_conv1", "enc_conv2+to_logits",
    "dec_conv1(composed)", "dec_conv2+to_params",
    "elbo_head", "finalize_loss", "to_params_dgrad", "dec_conv2_dgrad", "dec_conv1_dgrad(+logits_bwd, to_logits_dgrad if K<=4)",
    "logits_bwd(K>4)",
    "to_logits_dgrad(K>4)", "enc_conv2_dgrad", "to_params_wgrad", "dec_conv2_wgrad", "dec_conv1_wgrad",
    "to_logits_wgrad", "enc_conv2_wgrad", "enc_conv1_wgrad", "grad_tail(reduce_slabs+log_prior_grad)",
    "compose_bwd[+adam]", "(log_prior_grad: in grad_tail)"};

struct StepCtx {
  const float* const* w;
  const float* x;
  const float* u;
  int u_layout;
  const int64_t* lengths;
  const int64_t* norm;  // null or device {valid_count, batch} (kernels.h loss_norm_batch)
  float beta;
  int need_grad;    // 2: as 1, but the loss is finalized by the backward's tail launch (defer_loss)
  float* loss;
  double* loss_accum;
  const float* gscale;
  float* g;
  const AdamArgs* adam;  // non-null: Adam fused into the step's last launch (S_COMPOSE_BWD)
};

ConvArgs conv_of(const ElboPlan& p, const float* const* wp, int st) {
  static const float* const kNull[VQHMM_NPARAMS] = {};
  const float* const* w = wp ? wp : kNull;  // stage_work() only needs the shapes
  ConvArgs a = conv_base(p);
  a.Wimg = p.img[st];
  switch (st) {
    case S_ENC1:
      a.src = p.xp; a.Kc = p.D; a.ks = 3; a.W = w[ENC1_W]; a.bias = w[ENC1_B]; a.N = p.H; a.act = 1; a.out = p.h1e;
      break;
    case S_ENC2:
      a.src = p.h1e; a.Kc = p.H; a.ks = 3; a.W = w[ENC2_W]; a.bias = w[ENC2_B]; a.N = p.H2; a.act = 1; a.out = p.h2e;
      a.tW = w[LOGIT_W]; a.tb = w[LOGIT_B]; a.C2 = p.K; a.t_out = p.logits; a.q_out = p.q;
      break;
    case S_DEC1:
      a.src = p.q; a.Kc = p.K; a.ks = 3; a.W = p.Wc; a.bias = w[DEC1_B]; a.N = p.H; a.act = 1; a.out = p.g1;
      break;
    case S_DEC2:
      a.src = p.g1; a.Kc = p.H; a.ks = 3; a.W = w[DEC2_W]; a.bias = w[DEC2_B]; a.N = p.H; a.act = 1; a.out = p.g2;
      a.tW = w[PAR_W]; a.tb = w[PAR_B]; a.C2 = 2 * p.D; a.t_out = p.par;
      break;
    case S_PAR_DG:
      a.src = p.dpar; a.Kc = 2 * p.D; a.ks = 1; a.W = w[PAR_W]; a.w_dgrad = 1; a.N = p.H; a.act = 2; a.aux = p.g2;
      a.out = p.dg2;
      break;
    case S_DEC2_DG:
      a.src = p.dg2; a.Kc = p.H; a.ks = 3; a.W = w[DEC2_W]; a.w_dgrad = 1; a.N = p.H; a.act = 2; a.aux = p.g1;
      a.out = p.dg1;
      break;
    case S_DEC1_DG:
      a.src = p.dg1; a.Kc = p.H; a.ks = 3; a.W = p.Wc; a.w_dgrad = 1; a.N = p.K; a.act = 0; a.out = p.dqd;
      break;
    case S_LOGIT_DG:
      a.src = p.dlog; a.Kc = p.K; a.ks = 1; a.W = w[LOGIT_W]; a.w_dgrad = 1; a.N = p.H2; a.act = 2; a.aux = p.h2e;
      a.out = p.dh2;
      break;
    case S_ENC2_DG:
      a.src = p.dh2; a.Kc = p.H2; a.ks = 3; a.W = w[ENC2_W]; a.w_dgrad = 1; a.N = p.H; a.act = 2; a.aux = p.h1e;
      a.out = p.dh1;
      break;
  }
  return a;
}

// Convolutions whose conv2_kernel launches take a packed weight image (built once per step in
// the prologue, misc.hip wimg_slice) instead of re-packing W in every workgroup.
const int kImgStages[] = {S_ENC1, S_ENC2, S_DEC1, S_DEC2, S_PAR_DG, S_DEC2_DG, S_DEC1_DG, S_LOGIT_DG, S_ENC2_DG};

void plan_images(ElboPlan& p, Carver& c) {
  for (int st : kImgStages) {
    p.img[st] = nullptr;
    const ConvArgs a = conv_of(p, nullptr, st);
    if (conv2_supported(a)) p.img[st] = c.take<float>((size_t)c2_image_floats(a.N, a.Kc, a.ks));
  }
}

// The prologue's image jobs: each conv's effective weight, the composed decoder conv1
// (W' = W E^T, stages S_DEC1 / S_DEC1_DG) computed straight from W and E.
int image_jobs(const ElboPlan& p, const float* const* w, WImgJob* jobs) {
  int n = 0;
  for (int st : kImgStages) {
    if (!p.img[st]) continue;
    const ConvArgs a = conv_of(p, w, st);
    WImgJob j{};
    j.W = a.W; j.w_dgrad = a.w_dgrad; j.N = a.N; j.Kc = a.Kc; j.ks = a.ks; j.img = p.img[st];
    if (st == S_DEC1 || st == S_DEC1_DG) {
      j.composed = 1; j.W = w[DEC1_W]; j.E = w[EMB]; j.H = p.H;
    }
    jobs[n++] = j;
  }
  return n;
}

// Staged head: Prior MLP as 1x1 convs over PCL rows, L1/L2 row kernels, then the
// MLP backward as a dgrad conv + two wgrads (head_staged.hip).
int run_staged_head(const ElboPlan& p, const StepCtx& c, const float* const* w, hipStream_t s) {
  int rc;
  ConvArgs a = conv_base(p);
  a.src = p.up; a.Kc = p.U; a.ks = 1; a.W = w[TN0_W]; a.bias = w[TN0_B]; a.N = p.TH; a.act = 1; a.out = p.hid;
  if ((rc = launch_conv(a, s))) return rc;
  a = conv_base(p);
  a.src = p.hid; a.Kc = p.TH; a.ks = 1; a.W = w[TN2_W]; a.bias = w[TN2_B]; a.N = p.K * p.K; a.act = 0;
  a.out = p.lgA;
  if ((rc = launch_conv(a, s))) return rc;
  StagedHeadArgs h{};
  h.B = p.B; h.T = p.T; h.R = p.R; h.D = p.D; h.K = p.K;
  h.x = p.xp; h.par = p.par; h.logits = p.logits; h.q = p.q; h.lengths = c.lengths;
  h.log_prior = w[LOG_PRIOR]; h.log_pi = p.logpi; h.lgA = p.lgA; h.nx = p.nx; h.dqc = p.dqc; h.trw = p.trw;
  h.beta = c.beta; h.norm = c.norm; h.need_grad = c.need_grad;
  h.dpar = p.dpar; h.dlx = p.dlx; h.dqx = p.dqx; h.part = p.part; h.q0 = p.sq0;
  if ((rc = launch_staged_head(h, p.hgrid, s))) return rc;
  if (!c.need_grad) return VQHMM_OK;
  a = conv_base(p);
  a.src = p.lgA; a.Kc = p.K * p.K; a.ks = 1; a.W = w[TN2_W]; a.w_dgrad = 1; a.N = p.TH; a.act = 2; a.aux = p.hid;
  a.out = p.dhid;
  if ((rc = launch_conv(a, s))) return rc;
  const float* dys[2] = {p.dhid, p.lgA};
  const float* xs[2] = {p.up, p.hid};
  for (int i = 0; i < 2; ++i) {
    const WLayer& L = p.wl[6 + i];
    WgradArgs wa{};
    wa.dy = dys[i]; wa.x = xs[i]; wa.x_cf = 0; wa.R = p.R; wa.T = p.T;
    wa.N = L.N; wa.C = L.C; wa.ks = L.ks; wa.rows_per_chunk = L.rows; wa.slab = L.slab; wa.bias_slab = L.bslab;
    if ((rc = launch_wgrad(wa, s))) return rc;
  }
  return VQHMM_OK;
}

// The softmax backward (logits_bwd) rides in the dec_conv1 dgrad epilogue when that
// conv runs on conv2 and a row's K <= 8 channels sit in one or two lanes (ACT 3 / 4).
bool logits_bwd_fused(const ElboPlan& p) { return p.K <= 8 && conv2_supported(conv_of(p, nullptr, S_DEC1_DG)); }
// ... and to_logits' dgrad too when the encoder conv2 width splits into float4s over the 4 lane groups.
bool logits_dg_fused(const ElboPlan& p) { return logits_bwd_fused(p) && ld4(p.H2) % 16 == 0 && p.H2 <= 64; }

// The six convolutions' weight-gradient problems, in S_W_PAR .. S_W_ENC1 order (w: the parameters, for the
// composed layer's dE epilogue in the grouped launch).
void wgrad_jobs(const ElboPlan& p, const float* const* w, WgradArgs* wa) {
  const float* dys[6] = {p.dpar, p.dg2, p.dg1, p.dlog, p.dh2, p.dh1};
  const float* xs[6] = {p.g2, p.g1, p.q, p.h2e, p.h1e, p.xp};
  for (int i = 0; i < 6; ++i) {
    const WLayer& L = p.wl[i];
    wa[i] = WgradArgs{};
    wa[i].dy = dys[i]; wa[i].x = xs[i]; wa[i].x_cf = 0; wa[i].R = p.R; wa[i].T = p.T;
    wa[i].N = L.N; wa[i].C = L.C; wa[i].ks = L.ks; wa[i].rows_per_chunk = L.rows; wa[i].slab = L.slab;
    wa[i].bias_slab = L.bslab;
    static const bool no_cmp = VQHMM_PROF_ENV("VQHMM_WGRAD_NOCMP") != nullptr;  // timing only: dE left unwritten
    if (L.cslab && !no_cmp) {
      wa[i].cmpW = w[DEC1_W];
      wa[i].cmp_slab = L.cslab;
    }
  }
}

// The backward's slab segments (every weight gradient's per-chunk partials) for the tail launch.  Grouped
// weight gradients: the composed decoder conv1's dW is a composed segment over the dWc slab (its blocks
// reduce their own dWc rows) and its dE a plain segment over the per-chunk dE shares, so every parameter's
// gradient is complete after this one launch.  Otherwise the dWc segment reduces into p.dWc and the
// composed gradients follow in a second launch (compose_adam / compose_bwd).
void make_tail(const ElboPlan& p, const StepCtx& c, TailArgs& ta) {
  const float* const* w = c.w;
  int64_t off[VQHMM_NPARAMS + 1];
  vqhmm_dims_t d{p.D, p.H, p.K, p.H2, p.U, p.TH};
  vqhmm_param_layout(&d, off);
  float* g = c.g;
  const float* gs = c.gscale;
  int n = 0;
  auto seg = [&](const float* slab, int64_t nch, int64_t len, float* out, const float* scale) {
    ta.s[n++] = SlabSeg{slab, out, scale, nch, len, nullptr, 0, 0};
  };
  const WLayer* wl = p.wl;
  seg(wl[0].slab, wl[0].nchunks, (int64_t)wl[0].N * wl[0].C, g + off[PAR_W], gs);  // dpar is unscaled
  seg(wl[0].bslab, wl[0].nchunks, wl[0].N, g + off[PAR_B], gs);
  if (p.dec2_split) {  // two 32-output halves: [half][chunk][32][C][3], [half][chunk][32]
    const int64_t hw = (int64_t)32 * wl[1].C * 3;
    for (int h = 0; h < 2; ++h) {
      seg(wl[1].slab + h * wl[1].nchunks * hw, wl[1].nchunks, hw, g + off[DEC2_W] + h * hw, nullptr);
      seg(wl[1].bslab + h * wl[1].nchunks * 32, wl[1].nchunks, 32, g + off[DEC2_B] + h * 32, nullptr);
    }
  } else {
    seg(wl[1].slab, wl[1].nchunks, (int64_t)wl[1].N * wl[1].C * 3, g + off[DEC2_W], nullptr);
    if (p.wfold) { ta.s[n - 1].trO = wl[1].N; ta.s[n - 1].trC = wl[1].C; }  // the backward strip's row layout
    seg(wl[1].bslab, wl[1].nchunks, wl[1].N, g + off[DEC2_B], nullptr);
  }
  if (p.wgroup) {
    ta.s[n++] = SlabSeg{wl[2].slab, g + off[DEC1_W], nullptr, wl[2].nchunks, (int64_t)p.H * p.H * 3, p.Ecopy, p.H, p.K};
    seg(wl[2].cslab, wl[2].nchunks, (int64_t)p.K * p.H, g + off[EMB], nullptr);
  } else {
    seg(wl[2].slab, wl[2].nchunks, (int64_t)wl[2].N * wl[2].C * 3, p.dWc, nullptr);
  }
  seg(wl[2].bslab, wl[2].nchunks, wl[2].N, g + off[DEC1_B], nullptr);
  seg(wl[3].slab, wl[3].nchunks, (int64_t)wl[3].N * wl[3].C, g + off[LOGIT_W], nullptr);
  seg(wl[3].bslab, wl[3].nchunks, wl[3].N, g + off[LOGIT_B], nullptr);
  seg(wl[4].slab, wl[4].nchunks, (int64_t)wl[4].N * wl[4].C * 3, g + off[ENC2_W], nullptr);
  if (p.wfold) { ta.s[n - 1].trO = wl[4].N; ta.s[n - 1].trC = wl[4].C; }
  seg(wl[4].bslab, wl[4].nchunks, wl[4].N, g + off[ENC2_B], nullptr);
  seg(wl[5].slab, wl[5].nchunks, (int64_t)wl[5].N * wl[5].C * 3, g + off[ENC1_W], nullptr);
  seg(wl[5].bslab, wl[5].nchunks, wl[5].N, g + off[ENC1_B], nullptr);
  if (p.staged) {
    seg(wl[6].slab, wl[6].nchunks, (int64_t)p.TH * p.U, g + off[TN0_W], gs);
    seg(wl[6].bslab, wl[6].nchunks, p.TH, g + off[TN0_B], gs);
    seg(wl[7].slab, wl[7].nchunks, (int64_t)p.K * p.K * p.TH, g + off[TN2_W], gs);
    seg(wl[7].bslab, wl[7].nchunks, (int64_t)p.K * p.K, g + off[TN2_B], gs);
  } else {
    seg(p.sW1, p.hgrid, (int64_t)p.TH * p.U, g + off[TN0_W], gs);
    seg(p.sb1, p.hgrid, p.TH, g + off[TN0_B], gs);
    seg(p.sW2, p.hgrid, (int64_t)p.K * p.K * p.TH, g + off[TN2_W], gs);
    seg(p.sb2, p.hgrid, (int64_t)p.K * p.K, g + off[TN2_B], gs);
  }
  ta.nseg = n;
  ta.q0slab = p.sq0;
  ta.q0chunks = p.staged ? 1 : p.hgrid;
  ta.lp = LogPriorGradArgs{nullptr, w[LOG_PRIOR], p.K, c.beta, c.norm, p.B, c.gscale, g + off[LOG_PRIOR]};
  if (c.loss) {  // the forward ran with need_grad = 2
    ta.fin_part = p.part; ta.fin_nblk = p.hgrid; ta.fin_cnt = p.cnt; ta.fin_B = p.B; ta.fin_T = p.T;
    ta.fin_D = p.D; ta.fin_loss = c.loss; ta.fin_accum = c.loss_accum; ta.fin_pieces = p.pieces;
  }
}

// enc_conv1 -> enc_conv2, the composed dec_conv1 -> dec_conv2 and to_params_dgrad -> dec_conv2_dgrad
// as one launch each
// (conv2.hip conv2f_kernel); VQHMM_CONV_FUSE=0 keeps two launches (A/B), read once.
ConvArgs fused_pair(const ElboPlan& p, const float* const* w, int st) {
  ConvArgs a = conv_of(p, w, st);
  const ConvArgs f = conv_of(p, w, st - 1);
  a.src = f.src; a.f_Kc = f.Kc; a.f_ks = f.ks; a.f_act = f.act; a.f_Wimg = f.Wimg; a.f_bias = f.bias;
  a.f_aux = f.aux; a.f_out = f.out;
  return a;
}
bool front_fused(const ElboPlan& p, const float* const* w, int st) {
  static const bool on = [] {
    const char* e = VQHMM_ENV("VQHMM_CONV_FUSE");
    return !e || atoi(e) != 0;
  }();
  return on && (st == S_ENC2 || st == S_DEC2 || st == S_DEC2_DG) && conv2_fused_supported(fused_pair(p, w, st));
}

// The four forward convolutions as one strip launch (strip.hip) where its shapes apply; VQHMM_STRIP=0
// keeps the two pair launches (A/B), read once
bool strip_fwd_on(const ElboPlan& p) {
  return strip_fwd_env() && strip_fwd_supported(conv_of(p, nullptr, S_ENC1), conv_of(p, nullptr, S_ENC2),
                                   conv_of(p, nullptr, S_DEC1), conv_of(p, nullptr, S_DEC2));
}

// dec_conv1's data gradient with, for K <= 4, the softmax backward (+ to_logits' dgrad) in its epilogue
ConvArgs dec1_dg_args(const ElboPlan& p, const float* const* w, const float* gscale) {
  static const float* const kNull[VQHMM_NPARAMS] = {};
  if (!w) w = kNull;
  ConvArgs a = conv_of(p, w, S_DEC1_DG);
  if (logits_bwd_fused(p)) {  // + logits_bwd in the epilogue
    a.act = p.K <= 4 ? 3 : 4;
    a.lb_q = p.q; a.lb_dqx = p.dqx; a.lb_dlx = p.dlx; a.lb_scale = gscale; a.lb_dlog = p.dlog;
    if (logits_dg_fused(p)) {  // + to_logits_dgrad
      a.lb_W = w[LOGIT_W]; a.lb_h = p.h2e; a.lb_dh = p.dh2; a.lb_C = p.H2;
    }
  }
  return a;
}
// dec_conv1 dgrad -> enc_conv2 dgrad as one launch below 2^17 rows (conv2.hip conv2g_kernel);
// VQHMM_CONV_FUSE=0 switches it off too
bool bwd_pair_fused(const ElboPlan& p, const float* const* w, const float* gscale) {
  static const bool on = [] {
    const char* e = VQHMM_ENV("VQHMM_CONV_FUSE");
    return !e || atoi(e) != 0;
  }();
  // measured: a launch fewer wins at small batches (B = 128: 22.3 -> 16.8 us), break-even at B = 512,
  // and at cfg2 (207k rows) the two launches are 3 us faster (168 VGPRs + spills at 3 waves / SIMD;
  // 2 waves without spills: slower still).  VQHMM_BWD_PAIR_ROWS moves the threshold (A/B)
  static const int64_t max_rows = [] {
    const char* e = VQHMM_PROF_ENV("VQHMM_BWD_PAIR_ROWS");
    return e ? (int64_t)atoll(e) : (int64_t)1 << 17;
  }();
  if (!on || !logits_dg_fused(p) || p.R >= max_rows) return false;
  ConvArgs f = dec1_dg_args(p, w, gscale);
  if (!w) f.lb_dh = p.dh2;  // stage_info's shape-only query (any non-null marks the fused dgrad)
  return conv2_bwd_pair_supported(conv_of(p, w, S_ENC2_DG), f);
}

// The backward's four data-gradient convolutions as one strip launch (strip.hip) where its shapes apply;
// VQHMM_STRIP_BWD=0 keeps the pair launches (A/B), read once
// the backward strip's shape / switch conditions, without the row threshold
bool strip_bwd_shape_ok(const ElboPlan& p) {
  static const bool on = [] {
    const char* e = VQHMM_ENV("VQHMM_STRIP_BWD");
    return !e || atoi(e) != 0;
  }();
  return on && logits_dg_fused(p) &&
         strip_bwd_supported(conv_of(p, nullptr, S_PAR_DG), conv_of(p, nullptr, S_DEC2_DG), dec1_dg_args(p, nullptr, nullptr),
                             conv_of(p, nullptr, S_ENC2_DG));
}

// The six weight gradients folded into the backward strip (strip_bwdw.hip) at any row count: measured
// (tools/gpu_ab_rows.sh) cfg2 (207k rows) 0.4483 -> 0.4352 ms against the backward pair + grouped wgrad
bool strip_wfold_planned(const ElboPlan& p) {
  return strip_wgrad_env() && strip_bwd_shape_ok(p) &&
         strip_bwdw_supported(conv_of(p, nullptr, S_PAR_DG), conv_of(p, nullptr, S_DEC2_DG), dec1_dg_args(p, nullptr, nullptr),
                              conv_of(p, nullptr, S_ENC2_DG), p.D);
}

bool strip_bwd_on(const ElboPlan& p) {
  // measured (tools/gpu_stripab.sh): B = 128 0.124 -> 0.116 ms, 256 0.1765 -> 0.1715, 512 0.2784 -> 0.2761,
  // cfg2 (207k rows) 0.462 -> 0.467: without the folded weight gradients below 2^17 rows only, as the
  // backward pair; with them (p.wfold) at every row count
  static const int64_t max_rows = [] {  // A/B: VQHMM_STRIP_BWD_ROWS
    const char* e = VQHMM_PROF_ENV("VQHMM_STRIP_BWD_ROWS");
    return e ? (int64_t)atoll(e) : (int64_t)1 << 17;
  }();
  return (p.R < max_rows || p.wfold) && strip_bwd_shape_ok(p);
}

// VQHMM_TAIL_FUSED=0 (grouped weight gradients): the tail without Adam, then the Adam launch (A/B; the
// same bits); read once
bool tail_fused_on() {
  static const bool v = [] {
    const char* e = VQHMM_ENV("VQHMM_TAIL_FUSED");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// The Adam step counter of the fused tail (tail_kernel<true> applies Adam with the count some earlier launch of
// the same backward advanced: the grouped weight-gradient launch or the folded backward strip, workgroup 0), or
// null.  The one place that decides it, for the launch that advances the counter and the tail that applies it.
bool tail_applies_adam(const ElboPlan& p, const StepCtx& c) { return c.adam && p.wgroup && tail_fused_on(); }
int64_t* adam_step_inc(const ElboPlan& p, const StepCtx& c) { return tail_applies_adam(p, c) ? c.adam->step : nullptr; }

HeadArgs head_args(const ElboPlan& p, const StepCtx& c) {
  const float* const* w = c.w;
  HeadArgs h{};
  h.B = p.B; h.T = p.T; h.R = p.R; h.D = p.D; h.K = p.K; h.U = p.U; h.TH = p.TH;
  h.x = p.xp; h.u = p.up;
  h.lengths = c.lengths; h.par = p.par; h.logits = p.logits; h.q = p.q;
  h.W1 = w[TN0_W]; h.b1 = w[TN0_B]; h.W2 = w[TN2_W]; h.b2 = w[TN2_B]; h.log_prior = w[LOG_PRIOR];
  h.beta = c.beta; h.norm = c.norm; h.need_grad = c.need_grad;
  if (c.need_grad == 2 && !c.norm) h.cnt_in = p.cnt;  // the prologue counted the batch (S_TOPCL)
  h.dpar = p.dpar; h.dqx = p.dqx; h.dlx = p.dlx; h.part = p.part;
  h.slab_W1 = p.sW1; h.slab_b1 = p.sb1; h.slab_W2 = p.sW2; h.slab_b2 = p.sb2; h.slab_q0 = p.sq0;
  h.himg = p.himg;  // the prologue built it (S_TOPCL runs in every forward)
  return h;
}

int run_stage(const ElboPlan& p, const StepCtx& c, int st, hipStream_t s) {
  const float* const* w = c.w;
  switch (st) {
    case S_TOPCL: {  // x, u -> PCL and the composed decoder conv1 weight, one launch
      PrologueArgs a{};
      a.x = c.x; a.D = p.D; a.xsc = p.T; a.xst = 1; a.xp = p.xp;
      a.u = c.u; a.U = p.U; a.usc = c.u_layout == 0 ? p.T : 1; a.ust = c.u_layout == 0 ? 1 : p.U; a.up = p.up;
      a.B = p.B; a.T = p.T;
      a.W = w[DEC1_W]; a.E = w[EMB]; a.H = p.H; a.K = p.K; a.Wc = p.Wc;
      a.nimg = image_jobs(p, w, a.img);
      a.wc_img_f = p.img[S_DEC1];
      a.wc_img_d = p.img[S_DEC1_DG];
      a.Ecopy = p.Ecopy;
      a.Wcopy = p.Wcopy;
      if (c.need_grad == 2 && !c.norm) { a.lengths = c.lengths; a.cnt = p.cnt; }
      if (p.himg) {
        a.hW1 = w[TN0_W]; a.hb1 = w[TN0_B]; a.hW2 = w[TN2_W]; a.hTH = p.TH; a.himg = p.himg;
      }
      return launch_prologue(a, s);
    }
    case S_COMPOSE:  // runs inside S_TOPCL's launch
      return VQHMM_OK;
    case S_ENC1: case S_DEC1:
      if (strip_fwd_on(p)) return VQHMM_OK;            // in S_ENC2's strip launch
      if (front_fused(p, w, st + 1)) return VQHMM_OK;  // runs inside the next conv's launch
      return launch_conv(conv_of(p, w, st), s);
    case S_ENC2: case S_DEC2:
      if (strip_fwd_on(p)) {
        if (st == S_DEC2) return VQHMM_OK;
        const HeadArgs h = head_args(p, c);
        return launch_strip_fwd(conv_of(p, w, S_ENC1), conv_of(p, w, S_ENC2), conv_of(p, w, S_DEC1), conv_of(p, w, S_DEC2),
                                p.strip_head ? &h : nullptr, s);
      }
      if (p.strip_head) return VQHMM_EUNSUPPORTED;  // planned with the head in the strip: must not happen
      if (front_fused(p, w, st)) return launch_conv2_fused(fused_pair(p, w, st), s);
      return launch_conv(conv_of(p, w, st), s);
    case S_DEC2_DG:
      if (strip_bwd_on(p)) return VQHMM_OK;  // in S_ENC2_DG's strip launch
      if (front_fused(p, w, st)) {
        ConvArgs a = fused_pair(p, w, st);
        a.f_scale = c.gscale;  // the front is S_PAR_DG
        return launch_conv2_fused(a, s);
      }
      return launch_conv(conv_of(p, w, st), s);
    case S_ENC2_DG:
      if (strip_bwd_on(p)) {
        ConvArgs pd = conv_of(p, w, S_PAR_DG);
        pd.scale = c.gscale;  // dpar is the head's gradient for dloss = 1
        if (p.wfold) {  // + all six weight gradients (slab row per workgroup); advances the fused tail's Adam step
          StripWgradArgs sw{};
          sw.x = p.xp; sw.cmpW = w[DEC1_W];
          for (int i = 0; i < 6; ++i) {
            sw.slab[i] = p.wl[i].slab;
            sw.bslab[i] = p.wl[i].bslab;
          }
          sw.cslab = p.wl[2].cslab;
          sw.D = p.D; sw.K = p.K; sw.H2 = p.H2;
          sw.step_inc = adam_step_inc(p, c);
          return launch_strip_bwdw(pd, conv_of(p, w, S_DEC2_DG), dec1_dg_args(p, w, c.gscale), conv_of(p, w, st), sw, s);
        }
        return launch_strip_bwd(pd, conv_of(p, w, S_DEC2_DG), dec1_dg_args(p, w, c.gscale), conv_of(p, w, st), s);
      }
      if (bwd_pair_fused(p, w, c.gscale))
        return launch_conv2_bwd_pair(conv_of(p, w, st), dec1_dg_args(p, w, c.gscale), s);
      return launch_conv(conv_of(p, w, st), s);
    case S_LOGIT_DG:
      if (logits_dg_fused(p)) return VQHMM_OK;  // ran in S_DEC1_DG's epilogue
      return launch_conv(conv_of(p, w, st), s);
    case S_DEC1_DG: {
      if (strip_bwd_on(p) || bwd_pair_fused(p, w, c.gscale)) return VQHMM_OK;  // runs inside S_ENC2_DG's launch
      return launch_conv(dec1_dg_args(p, w, c.gscale), s);
    }
    case S_PAR_DG: {
      if (strip_bwd_on(p) || front_fused(p, w, S_DEC2_DG)) return VQHMM_OK;  // in a later stage's launch
      ConvArgs a = conv_of(p, w, st);
      a.scale = c.gscale;  // dpar is the head's gradient for dloss = 1
      return launch_conv(a, s);
    }
    case S_HEAD: {
      if (p.staged) return run_staged_head(p, c, w, s);
      if (p.strip_head) return VQHMM_OK;  // in S_ENC2's strip launch
      const HeadArgs h = head_args(p, c);
      if (p.pipe_head) return launch_head_pipe(h, p.hgrid, s);
      if (p.coop_head) return launch_head_coop(h, p.hgrid, s);
      return launch_head(h, p.hgrid, s);
    }
    case S_FINAL:
      if (c.need_grad == 2) return VQHMM_OK;  // the backward's tail launch finalizes the loss
      return launch_finalize_loss(p.part, p.hgrid, c.lengths, c.norm, p.B, p.T, p.D, c.beta, c.loss, c.loss_accum,
                                  p.pieces, s);
    case S_LOGIT_BWD:
      if (logits_bwd_fused(p)) return VQHMM_OK;  // ran in S_DEC1_DG's epilogue
      return launch_logits_bwd(p.q, p.dqd, p.dqx, p.dlx, c.gscale, p.R, p.K, p.dlog, s);
    case S_W_PAR: case S_W_DEC2: case S_W_DEC1: case S_W_LOGIT: case S_W_ENC2: case S_W_ENC1: {
      if (p.wfold) return VQHMM_OK;  // in S_ENC2_DG's backward strip launch
      WgradArgs wa[6];
      wgrad_jobs(p, w, wa);
      if (p.wgroup) {  // all six in S_W_ENC1's launch (every dY is ready by then, in any stage order)
        if (st != S_W_ENC1) return VQHMM_OK;
        // timing experiment only (gradients are then incomplete): VQHMM_WGRAD_JOBMASK bit i keeps job i
        static const int jmask = [] {
          const char* e = VQHMM_PROF_ENV("VQHMM_WGRAD_JOBMASK");
          return e ? atoi(e) : 63;
        }();
        if (jmask != 63) {
          WgradArgs sel[6];
          int n = 0;
          for (int i = 0; i < 6; ++i)
            if (jmask >> i & 1) sel[n++] = wa[i];
          return n ? launch_wgrad2_group(sel, n, s, adam_step_inc(p, c)) : VQHMM_OK;
        }
        // the fused tail applies Adam without a completion ticket: this launch advances the step counter
        int64_t* step_inc = adam_step_inc(p, c);
        if (p.dec2_split) {
          WgradArgs sp[7];
          int n = 0;
          for (int i = 0; i < 6; ++i) {
            if (i != 1) {
              sp[n++] = wa[i];
              continue;
            }
            const WLayer& L = p.wl[1];
            for (int h = 0; h < 2; ++h) {
              WgradArgs hw = wa[1];
              hw.dy = wa[1].dy + 32 * h;
              hw.ld_dy = ld4(L.N);
              hw.N = 32;
              hw.slab = L.slab + (int64_t)h * L.nchunks * 32 * L.C * L.ks;
              hw.bias_slab = L.bslab + (int64_t)h * L.nchunks * 32;
              sp[n++] = hw;
            }
          }
          return launch_wgrad2_group(sp, n, s, step_inc);
        }
        return launch_wgrad2_group(wa, 6, s, step_inc);
      }
      return launch_wgrad(wa[st - S_W_PAR], s);
    }
    case S_REDUCE: {
      if (p.wgroup && tail_fused_on()) return VQHMM_OK;  // in S_COMPOSE_BWD's launch (tail_kernel)
      TailArgs ta{};
      make_tail(p, c, ta);
      return launch_grad_tail(ta, s);
    }
    case S_COMPOSE_BWD: {
      int64_t off[VQHMM_NPARAMS + 1];
      vqhmm_dims_t d{p.D, p.H, p.K, p.H2, p.U, p.TH};
      vqhmm_param_layout(&d, off);
      if (p.wgroup) {  // every gradient is complete after the tail launch
        if (tail_fused_on()) {  // slab reduction (+ Adam on each reduced column) in one launch
          TailArgs ta{};
          make_tail(p, c, ta);
          return launch_tail(ta, tail_applies_adam(p, c) ? c.adam : nullptr, c.g, s);
        }
        if (!c.adam) return VQHMM_OK;
        const AdamArgs& ad = *c.adam;
        return launch_adam(ad.p, c.g, ad.m, ad.v, off[VQHMM_NPARAMS], ad.lr, ad.b1, ad.b2, ad.eps, ad.step, ad.gmul, s);
      }
      ComposeAdamArgs ca{};
      ca.dWc = p.dWc; ca.H = p.H; ca.K = p.K;
      ca.g = c.g; ca.n = off[VQHMM_NPARAMS]; ca.off_w = off[DEC1_W]; ca.off_e = off[EMB];
      if (c.adam) {  // this launch updates the parameters: E / W from the prologue's copies
        ca.Ecopy = p.Ecopy; ca.Wcopy = p.Wcopy;
        ca.adam = *c.adam;
        return launch_compose_adam(ca, s);
      }
      const LogPriorGradArgs lp{nullptr, nullptr, p.K, c.beta, c.norm, p.B, c.gscale, nullptr};  // in S_REDUCE
      return launch_compose_bwd(p.dWc, w[DEC1_W], w[EMB], p.H, p.K, c.g + off[DEC1_W], c.g + off[EMB], lp, s);
    }
    case S_LOGPRIOR:  // runs inside S_COMPOSE_BWD's launch
      return VQHMM_OK;
  }
  return VQHMM_EINVAL;
}

// Algorithmic work of one launch of a stage (what roofline.achieved is computed from).
void stage_work(const ElboPlan& p, int st, double* flops, double* bytes, int* mfma) {
  const double N = (double)p.B * p.T;  // valid positions
  const double R = (double)p.R;
  *flops = 0; *bytes = 0; *mfma = 0;
  if (st == S_ENC1 || st == S_ENC2 || st == S_DEC1 || st == S_DEC2 || st == S_PAR_DG || st == S_DEC2_DG ||
      st == S_DEC1_DG || st == S_LOGIT_DG || st == S_ENC2_DG) {
    ConvArgs a = conv_of(p, nullptr, st);
    *flops = 2.0 * N * a.N * a.Kc * a.ks + (a.tW ? 2.0 * N * a.C2 * a.N : 0.0);
    *bytes = 4.0 * (R * a.Kc + R * a.N + (a.act == 2 ? R * a.N : 0) + (a.tW ? R * a.C2 * (a.q_out ? 2 : 1) : 0));
    *mfma = 1;
  } else if (st >= S_W_PAR && st <= S_W_ENC1) {
    const int i0 = p.wgroup ? 0 : st - S_W_PAR, i1 = p.wgroup ? (st == S_W_ENC1 ? 6 : 0) : i0 + 1;
    for (int i = i0; i < i1; ++i) {  // grouped: S_W_ENC1's launch does all six
      const WLayer& L = p.wl[i];
      *flops += 2.0 * N * L.N * L.C * L.ks;
      *bytes += 4.0 * (R * L.N + R * L.C + (double)L.nchunks * (L.N * L.C * L.ks + L.N));
    }
    *mfma = 1;
  } else if (st == S_HEAD) {
    const double KK = (double)p.K * p.K;
    // Prior MLP fwd (2 TH U + 2 TH K^2) + bwd (dh 2 TH K^2, dW2 2 TH K^2, dW1 2 TH U) + elementwise
    *flops = N * (4.0 * p.TH * p.U + 6.0 * p.TH * KK + 20.0 * p.D + 12.0 * KK);
    *bytes = 4.0 * R * (2 * p.D + p.D + p.U + 2 * p.K + 2 * p.D + 2 * p.K);
    HeadArgs h{};
    h.K = p.K; h.U = p.U; h.TH = p.TH; h.D = p.D; h.R = p.R;
    // the staged head (K > 8) is its Prior MLP's dense contractions on the wide conv / wgrad kernels (MFMA)
    *mfma = (head_mfma_supported(h) || head_coop_supported(h) || p.staged) ? 1 : 0;
  } else if (st == S_TOPCL) {
    *bytes = 4.0 * (N * (p.D + p.U) + R * (ld4(p.D) + ld4(p.U)));
  } else if (st == S_LOGIT_BWD) {
    *bytes = 4.0 * R * 6 * p.K;
    *flops = R * 8.0 * p.K;
  } else if (st == S_REDUCE) {
    double b = 0;
    for (int i = 0; i < 6; ++i)
      b += (double)p.wl[i].nchunks * (p.wl[i].N * p.wl[i].C * p.wl[i].ks + p.wl[i].N + (p.wl[i].cslab ? p.K * p.H : 0));
    b += (double)p.hgrid * ((double)p.TH * p.U + p.TH + (double)p.K * p.K * p.TH + p.K * p.K + p.K);
    *bytes = 4.0 * b;
    *flops = b;
  }
}

}  // namespace

extern "C" {

int vqhmm_elbo_fwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const float* u, int u_layout,
                       const int64_t* lengths, const int64_t* norm, int64_t B, int64_t T, float beta, int need_grad,
                       void* ws, size_t ws_bytes, float* loss, double* loss_accum, void* stream) {
  if (!dims_ok(d) || !w || B <= 0 || T <= 0 || !x || !u || !lengths || !ws || !loss || need_grad < 0 ||
      need_grad > 2)
    return VQHMM_EINVAL;
  for (int i = 0; i < VQHMM_NPARAMS; ++i)
    if (!w[i]) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  StepCtx c{w, x, u, u_layout, lengths, norm, beta, need_grad, loss, loss_accum, nullptr, nullptr, nullptr};
  for (int st = FWD_FIRST; st <= FWD_LAST; ++st)
    if (int rc = run_stage(p, c, st, (hipStream_t)stream)) return rc;
  return VQHMM_OK;
}

int vqhmm_elbo_bwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const int64_t* norm, int64_t B,
                       int64_t T, float beta, const float* grad_scale, void* ws, size_t ws_bytes, float* g,
                       void* stream) {
  if (!dims_ok(d) || !w || B <= 0 || T <= 0 || !x || !ws || !g) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  StepCtx c{w, x, nullptr, 0, nullptr, norm, beta, 1, nullptr, nullptr, grad_scale, g, nullptr};
  for (int st = BWD_FIRST; st <= BWD_LAST; ++st)
    if (int rc = run_stage(p, c, st, (hipStream_t)stream)) return rc;
  return VQHMM_OK;
}

int vqhmm_elbo_bwd_loss_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const int64_t* norm,
                            int64_t B, int64_t T, float beta, const float* grad_scale, void* ws, size_t ws_bytes,
                            float* g, float* loss, double* loss_accum, void* stream) {
  if (!dims_ok(d) || !w || B <= 0 || T <= 0 || !x || !ws || !g || !loss) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  StepCtx c{w, x, nullptr, 0, nullptr, norm, beta, 1, loss, loss_accum, grad_scale, g, nullptr};
  for (int st = BWD_FIRST; st <= BWD_LAST; ++st)  // the tail launch finalizes the loss (make_tail: c.loss)
    if (int rc = run_stage(p, c, st, (hipStream_t)stream)) return rc;
  return VQHMM_OK;
}

int vqhmm_elbo_bwd_adam_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const int64_t* norm,
                            int64_t B, int64_t T, float beta, void* ws, size_t ws_bytes, float* g, float* param,
                            float* exp_avg, float* exp_avg_sq, double lr, double beta1, double beta2, double eps,
                            int64_t* step, float grad_scale, float* loss, double* loss_accum, void* stream) {
  if (!dims_ok(d) || !w || B <= 0 || T <= 0 || !x || !ws || !g || !param || !exp_avg || !exp_avg_sq || !step)
    return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  int64_t off[VQHMM_NPARAMS + 1];
  vqhmm_param_layout(d, off);
  for (int i = 0; i < VQHMM_NPARAMS; ++i)  // the last launch updates param in place: w must be its views
    if (w[i] != param + off[i]) return VQHMM_EINVAL;
  AdamArgs ad{param, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps, grad_scale};
  StepCtx c{w, x, nullptr, 0, nullptr, norm, beta, 1, loss, loss_accum, nullptr, g, &ad};
  for (int st = BWD_FIRST; st <= BWD_LAST; ++st)
    if (int rc = run_stage(p, c, st, (hipStream_t)stream)) return rc;
  return VQHMM_OK;
}

int vqhmm_elbo_num_stages(void) { return S_COUNT; }

int vqhmm_elbo_stage_info(const vqhmm_dims_t* d, int64_t B, int64_t T, int stage, char* name, size_t name_len,
                          double* flops, double* bytes, int* mfma_bound) {
  if (!dims_ok(d) || stage < 0 || stage >= S_COUNT || B <= 0 || T <= 0) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, nullptr);
  // fused conv pairs: decided on a plan with (never dereferenced) workspace addresses
  const int pair_of = stage == S_ENC1 ? S_ENC2 : stage == S_DEC1 ? S_DEC2 : stage == S_PAR_DG ? S_DEC2_DG : stage;
  const bool fused_front = (pair_of == S_ENC2 || pair_of == S_DEC2 || pair_of == S_DEC2_DG) &&
                           front_fused(plan_elbo(d, B, T, reinterpret_cast<void*>(4096)), nullptr, pair_of);
  const bool bwd_pair = bwd_pair_fused(plan_elbo(d, B, T, reinterpret_cast<void*>(4096)), nullptr, nullptr);
  const bool strip = strip_fwd_on(plan_elbo(d, B, T, reinterpret_cast<void*>(4096)));
  const bool in_strip = strip && (stage == S_ENC1 || stage == S_ENC2 || stage == S_DEC1 || stage == S_DEC2 ||
                                   (p.strip_head && stage == S_HEAD));
  const bool bstrip = strip_bwd_on(plan_elbo(d, B, T, reinterpret_cast<void*>(4096)));
  const bool in_bstrip = bstrip && (stage == S_PAR_DG || stage == S_DEC2_DG || stage == S_DEC1_DG ||
                                    stage == S_LOGIT_BWD || stage == S_LOGIT_DG || stage == S_ENC2_DG);
  if (name && name_len) {
    const char* nm = kStageNames[stage];
    if (in_strip)
      nm = stage != S_ENC2 ? "(in strip_fwd)"
           : p.strip_head ? "strip_fwd(enc_conv1+enc_conv2+to_logits+dec_conv1+dec_conv2+to_params+elbo_head)"
                          : "strip_fwd(enc_conv1+enc_conv2+to_logits+dec_conv1+dec_conv2+to_params)";
    if (p.strip_head && stage == S_HEAD) nm = "(elbo_head: in strip_fwd)";
    if (in_bstrip)
      nm = stage != S_ENC2_DG ? "(in strip_bwd)"
           : p.wfold ? "strip_bwdw(to_params_dgrad+dec_conv2_dgrad+dec_conv1_dgrad+logits_bwd+to_logits_dgrad+enc_conv2_dgrad+6 wgrads)"
                     : "strip_bwd(to_params_dgrad+dec_conv2_dgrad+dec_conv1_dgrad+logits_bwd+to_logits_dgrad+enc_conv2_dgrad)";
    if (p.wfold && stage >= S_W_PAR && stage <= S_W_ENC1) nm = "(wgrad: in strip_bwdw)";
    else if (p.wgroup && stage == S_W_ENC1) nm = "wgrad_group(all 6 weight gradients)";
    else if (p.wgroup && stage >= S_W_PAR && stage < S_W_ENC1) nm = "(wgrad: in wgrad_group)";
    else if (in_strip || in_bstrip || (p.strip_head && stage == S_HEAD)) {
    } else if (fused_front && (stage == S_ENC1 || stage == S_DEC1 || stage == S_PAR_DG))
      nm = stage == S_ENC1 ? "(enc_conv1: in enc_conv2's launch)"
           : stage == S_DEC1 ? "(dec_conv1: in dec_conv2's launch)" : "(to_params_dgrad: in dec_conv2_dgrad's launch)";
    else if (fused_front && stage == S_ENC2) nm = "enc_conv1+enc_conv2+to_logits";
    else if (fused_front && stage == S_DEC2) nm = "dec_conv1+dec_conv2+to_params";
    else if (fused_front && stage == S_DEC2_DG) nm = "to_params_dgrad+dec_conv2_dgrad";
    else if (bwd_pair && stage == S_DEC1_DG) nm = "(dec_conv1_dgrad: in enc_conv2_dgrad's launch)";
    else if (bwd_pair && stage == S_ENC2_DG) nm = "dec_conv1_dgrad+logits_bwd+to_logits_dgrad+enc_conv2_dgrad";
    else if (stage == S_LOGIT_BWD && logits_bwd_fused(p)) nm = "(logits_bwd: in dec_conv1_dgrad's epilogue)";
    else if (stage == S_LOGIT_DG && logits_dg_fused(p)) nm = "(to_logits_dgrad: in dec_conv1_dgrad's epilogue)";
    else if (p.wgroup && tail_fused_on() && stage == S_REDUCE) nm = "(grad_tail: in the tail launch)";
    else if (p.wgroup && tail_fused_on() && stage == S_COMPOSE_BWD) nm = "tail(slab reduction+composed dW/dE[+adam])";
    else if (p.wgroup && stage == S_REDUCE) nm = "grad_tail(slab reduction+composed dW/dE)";
    else if (p.wgroup && stage == S_COMPOSE_BWD) nm = "[adam]";
    strncpy(name, nm, name_len - 1);
    name[name_len - 1] = 0;
  }
  double f, b;
  int m;
  stage_work(p, stage, &f, &b, &m);
  if (in_strip) {  // S_ENC2's launch does all four; HBM sees x in and every activation out once
    f = 0; b = 0;
    if (stage == S_ENC2) {
      for (int st2 : {S_ENC1, S_ENC2, S_DEC1, S_DEC2}) {
        double f1, b1;
        int m1;
        stage_work(p, st2, &f1, &b1, &m1);
        f += f1;
      }
      const double R = (double)p.R;
      b = 4.0 * R * (ld4(p.D) + ld4(p.H) + ld4(p.H2) + 2 * ld4(p.K) + 2 * ld4(p.H) + ld4(2 * p.D));
      if (p.strip_head) {  // + the head: its flops; HBM: u in, dpar / dqx / dlx out (its other inputs are on chip)
        double f1, b1;
        int m1;
        stage_work(p, S_HEAD, &f1, &b1, &m1);
        f += f1;
        b += 4.0 * R * (ld4(p.U) + ld4(2 * p.D) + 2 * ld4(p.K));
      }
    }
  } else if (in_bstrip) {  // S_ENC2_DG's launch does all six; HBM: dpar, the masks, q / dqx / dlx, h2 in, grads out
    f = 0; b = 0;
    if (stage == S_ENC2_DG) {
      for (int st2 : {S_PAR_DG, S_DEC2_DG, S_DEC1_DG, S_LOGIT_BWD, S_LOGIT_DG, S_ENC2_DG}) {
        double f1, b1;
        int m1;
        stage_work(p, st2, &f1, &b1, &m1);
        f += f1;
      }
      const double R = (double)p.R;
      if (!p.wfold) {
        b = 4.0 * R * (ld4(2 * p.D) + 3 * ld4(p.H) + 3 * ld4(p.K) + ld4(p.H2) +          // dpar, g2, g1, h1, q, dqx, dlx, h2
                       2 * ld4(p.H) + 2 * ld4(p.K) + ld4(p.H2) + ld4(p.H));             // dg2, dg1, dqd, dlog, dh2, dh1
      } else {  // + the six weight gradients: x in, the dY never leave the chip, one slab row per workgroup out
        double fw, bw;
        int mw;
        stage_work(p, S_W_ENC1, &fw, &bw, &mw);
        f += fw;
        b = 4.0 * R * (ld4(2 * p.D) + 3 * ld4(p.H) + 3 * ld4(p.K) + ld4(p.H2) + ld4(p.D));
        for (int i = 0; i < 6; ++i)
          b += 4.0 * p.wl[i].nchunks * ((double)p.wl[i].N * p.wl[i].C * p.wl[i].ks + p.wl[i].N);
        b += 4.0 * p.wl[2].nchunks * (double)p.K * p.H;
      }
    }
  } else if (p.wfold && stage >= S_W_PAR && stage <= S_W_ENC1) {
    f = 0; b = 0;  // counted with the backward strip
  } else if (fused_front && pair_of != stage) {
    f = 0; b = 0;  // counted with the launch it runs in
  } else if (fused_front) {
    double f1, b1;
    int m1;
    stage_work(p, stage == S_ENC2 ? S_ENC1 : stage == S_DEC2 ? S_DEC1 : S_PAR_DG, &f1, &b1, &m1);
    f += f1;
    b += b1;
  }
  if (in_bstrip) {
  } else if ((stage == S_LOGIT_BWD && logits_bwd_fused(p)) || (stage == S_LOGIT_DG && logits_dg_fused(p))) {
    f = 0; b = 0;
  } else if (stage == S_DEC1_DG && logits_bwd_fused(p)) {  // its epilogue does the logits backward (+ dgrad)
    double f1, b1;
    int m1;
    stage_work(p, S_LOGIT_BWD, &f1, &b1, &m1);
    f += f1;
    b += b1;
    if (logits_dg_fused(p)) {
      stage_work(p, S_LOGIT_DG, &f1, &b1, &m1);
      f += f1;
      b += b1;
    }
    m = 0;  // K output channels: bytes, not flops, bound it
  }
  if (in_bstrip) {
  } else if (bwd_pair && stage == S_DEC1_DG) {
    f = 0; b = 0;
  } else if (bwd_pair && stage == S_ENC2_DG) {  // + dec_conv1 dgrad with its fused epilogue work
    double f1, b1;
    int m1;
    stage_work(p, S_DEC1_DG, &f1, &b1, &m1);
    f += f1; b += b1;
    stage_work(p, S_LOGIT_BWD, &f1, &b1, &m1);
    f += f1; b += b1;
    stage_work(p, S_LOGIT_DG, &f1, &b1, &m1);
    f += f1; b += b1;
  }
  if (p.wgroup && tail_fused_on() && stage == S_REDUCE) {
    f = 0; b = 0;
  } else if (p.wgroup && tail_fused_on() && stage == S_COMPOSE_BWD) {
    double f1, b1;
    int m1;
    stage_work(p, S_REDUCE, &f1, &b1, &m1);
    f += f1;
    b += b1;
  }
  if (flops) *flops = f;
  if (bytes) *bytes = b;
  if (mfma_bound) *mfma_bound = m;
  return VQHMM_OK;
}

int vqhmm_elbo_stage_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const float* u, int u_layout,
                         const int64_t* lengths, const int64_t* norm, int64_t B, int64_t T, float beta, void* ws,
                         size_t ws_bytes, float* grad, int stage, void* stream) {
  if (!dims_ok(d) || !w || !ws || stage < 0 || stage >= S_COUNT) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  StepCtx c{w, x, u, u_layout, lengths, norm, beta, 1, p.loss, nullptr, nullptr, grad, nullptr};
  return run_stage(p, c, stage, (hipStream_t)stream);
}

int vqhmm_elbo_pieces(const vqhmm_dims_t* d, int64_t B, int64_t T, const void* ws, const float** loss,
                      const float** pieces) {
  if (!dims_ok(d) || !ws) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, const_cast<void*>(ws));
  if (loss) *loss = p.loss;
  if (pieces) *pieces = p.pieces;
  return VQHMM_OK;
}

int vqhmm_elbo_status_offset(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* offset) {
  if (!dims_ok(d) || B <= 0 || T <= 0 || !offset) return VQHMM_EINVAL;
  // a plan on a non-null base: only the carved offsets are used, nothing is dereferenced
  char* const base = reinterpret_cast<char*>(4096);
  const ElboPlan p = plan_elbo(d, B, T, base);
  *offset = (size_t)(reinterpret_cast<char*>(p.sync + 2) - base);
  return VQHMM_OK;
}

int vqhmm_elbo_debug_buffers(const vqhmm_dims_t* d, int64_t B, int64_t T, const void* ws, const float** out) {
  if (!dims_ok(d) || !ws || !out) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, const_cast<void*>(ws));
  const float* v[16] = {p.xp, p.h1e, p.h2e, p.logits, p.q, p.g1, p.g2, p.par,
                        p.dpar, p.dg2, p.dg1, p.dqd, p.dlog, p.dh2, p.dh1, p.dqx};
  for (int i = 0; i < 16; ++i) out[i] = v[i];
  return VQHMM_OK;
}

int vqhmm_debug_prof(int which, uint64_t* out, int64_t n) {
  if (!out || n < 0 || n > 256 * 16) return VQHMM_EINVAL;
  switch (which) {
    case 0: return strip_prof_copy(out, n);
    case 1: return conv2_prof_copy(out, n);
    case 2: return head_prof_copy(out, n);
    case 3: return bwdw_prof_copy(out, n);
  }
  return VQHMM_EINVAL;
}

int vqhmm_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                   double beta1, double beta2, double eps, int64_t* step, float grad_scale, void* stream) {
  if (n < 0 || !step || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq))) return VQHMM_EINVAL;
  return launch_adam(param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, step, grad_scale,
                     (hipStream_t)stream);
}

int vqhmm_clip_grad_norm_f32(float* grad, int64_t n, float pre_scale, float max_norm, float* total_norm,
                              void* stream) {
  if (n < 0 || (n > 0 && !grad) || !(max_norm > 0.f)) return VQHMM_EINVAL;
  return launch_clip_grad_norm(grad, n, pre_scale, max_norm, total_norm, (hipStream_t)stream);
}

int vqhmm_gather_chunks_f32(const float* src, const int64_t* meta, int64_t B, int64_t C, int64_t Tmax, float* out,
                            void* stream) {
  if (B < 0 || C < 0 || Tmax < 0 || C > INT32_MAX || Tmax > INT32_MAX) return VQHMM_EINVAL;
  if (B * C * Tmax > 0 && (!src || !meta || !out)) return VQHMM_EINVAL;
  return launch_gather_chunks(src, meta, B, C, Tmax, out, (hipStream_t)stream);
}

// ---------------------------------------------------------------- inference surface
int vqhmm_infer_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* bytes) {
  if (!dims_ok(d) || B < 0 || T < 0 || !bytes) return VQHMM_EINVAL;
  const int64_t R = B * (T + 2);
  const int hw = ld4(d->hidden_dim > d->hidden_dim2 ? d->hidden_dim : d->hidden_dim2);
  Carver c{nullptr};
  c.take<float>(R * hw);
  c.take<float>(R * hw);
  c.take<float>(R * ld4(d->K));
  c.take<float>(R * ld4(d->input_dim > d->K ? d->input_dim : d->K));
  c.take<float>((size_t)d->hidden_dim * d->K * 3);
  *bytes = c.off + 256;
  return VQHMM_OK;
}

// x is CF (B, D, T); it is first copied into the padded PCL buffer xin.
static int encode_impl(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int64_t T,
                       float* logits_cf, float* q_cf, float* q_pcl, float* xin, float* bufA, float* bufB,
                       hipStream_t s, int32_t* regimes = nullptr) {
  const int64_t R = B * (T + 2);
  int rc;
  if ((rc = launch_to_pcl(x, d->input_dim, B, (int)T, T, 1, xin, s))) return rc;
  ConvArgs a{};
  a.R = R; a.T = (int)T;
  a.src = xin; a.Kc = d->input_dim; a.ks = 3; a.W = w[ENC1_W]; a.bias = w[ENC1_B];
  a.N = d->hidden_dim; a.act = 1; a.out = bufA;
  if ((rc = launch_conv(a, s))) return rc;
  a = ConvArgs{};
  a.R = R; a.T = (int)T;
  a.src = bufA; a.Kc = d->hidden_dim; a.ks = 3; a.W = w[ENC2_W]; a.bias = w[ENC2_B]; a.N = d->hidden_dim2;
  a.act = 1; a.out = bufB;
  a.tW = w[LOGIT_W]; a.tb = w[LOGIT_B]; a.C2 = d->K;
  if (logits_cf) { a.t_cf0 = logits_cf; a.t_split = d->K; }
  a.q_out = q_pcl;
  a.q_cf = q_cf;
  a.reg_out = regimes;
  if (logits_cf && (q_cf || regimes)) return VQHMM_EINVAL;
  return launch_conv(a, s);
}

// q is either CF (B, K, T) (q_cf = 1: copied into the PCL buffer qin first) or
// already PCL (q_cf = 0, q == qin).
static int decode_impl(const vqhmm_dims_t* d, const float* const* w, const float* q, int q_cf, int64_t B,
                       int64_t T, float* mu, float* logvar, float* qin, float* bufA, float* bufB, float* Wc,
                       hipStream_t s) {
  const int64_t R = B * (T + 2);
  int rc;
  if ((rc = launch_compose_fwd(w[DEC1_W], w[EMB], d->hidden_dim, d->K, Wc, s))) return rc;
  if (q_cf && (rc = launch_to_pcl(q, d->K, B, (int)T, T, 1, qin, s))) return rc;
  ConvArgs a{};
  a.R = R; a.T = (int)T;
  a.src = qin; a.Kc = d->K; a.ks = 3; a.W = Wc; a.bias = w[DEC1_B]; a.N = d->hidden_dim;
  a.act = 1; a.out = bufA;
  if ((rc = launch_conv(a, s))) return rc;
  a = ConvArgs{};
  a.R = R; a.T = (int)T;
  a.src = bufA; a.Kc = d->hidden_dim; a.ks = 3; a.W = w[DEC2_W]; a.bias = w[DEC2_B]; a.N = d->hidden_dim;
  a.act = 1; a.out = bufB;
  a.tW = w[PAR_W]; a.tb = w[PAR_B]; a.C2 = 2 * d->input_dim; a.t_cf0 = mu; a.t_cf1 = logvar;
  a.t_split = d->input_dim;
  return launch_conv(a, s);
}

struct InferBufs { float *A, *B, *q, *in, *Wc; };
static InferBufs carve_infer(const vqhmm_dims_t* d, int64_t B, int64_t T, void* ws) {
  const int64_t R = B * (T + 2);
  const int hw = ld4(d->hidden_dim > d->hidden_dim2 ? d->hidden_dim : d->hidden_dim2);
  Carver c{reinterpret_cast<char*>(ws)};
  InferBufs b;
  b.A = c.take<float>(R * hw);
  b.B = c.take<float>(R * hw);
  b.q = c.take<float>(R * ld4(d->K));
  b.in = c.take<float>(R * ld4(d->input_dim > d->K ? d->input_dim : d->K));
  b.Wc = c.take<float>((size_t)d->hidden_dim * d->K * 3);
  return b;
}

int vqhmm_encode_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int64_t T,
                     float* logits, void* ws, size_t ws_bytes, void* stream) {
  if (!dims_ok(d) || !w || !x || !logits || !ws || B < 0 || T < 0) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  size_t need;
  vqhmm_infer_workspace_size(d, B, T, &need);
  if (ws_bytes < need) return VQHMM_EWORKSPACE;
  InferBufs b = carve_infer(d, B, T, ws);
  return encode_impl(d, w, x, B, T, logits, nullptr, nullptr, b.in, b.A, b.B, (hipStream_t)stream);
}

int vqhmm_decode_f32(const vqhmm_dims_t* d, const float* const* w, const float* q, int64_t B, int64_t T, float* mu,
                     float* logvar, void* ws, size_t ws_bytes, void* stream) {
  if (!dims_ok(d) || !w || !q || !mu || !logvar || !ws || B < 0 || T < 0) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  size_t need;
  vqhmm_infer_workspace_size(d, B, T, &need);
  if (ws_bytes < need) return VQHMM_EWORKSPACE;
  InferBufs b = carve_infer(d, B, T, ws);
  return decode_impl(d, w, q, 1, B, T, mu, logvar, b.in, b.A, b.B, b.Wc, (hipStream_t)stream);
}

int vqhmm_forward_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int64_t T, float* mu,
                      float* logvar, float* q, void* ws, size_t ws_bytes, void* stream) {
  if (!dims_ok(d) || !w || !x || !mu || !logvar || !q || !ws || B < 0 || T < 0) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  size_t need;
  vqhmm_infer_workspace_size(d, B, T, &need);
  if (ws_bytes < need) return VQHMM_EWORKSPACE;
  InferBufs b = carve_infer(d, B, T, ws);
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = encode_impl(d, w, x, B, T, nullptr, q, b.q, b.in, b.A, b.B, s))) return rc;
  return decode_impl(d, w, b.q, 0, B, T, mu, logvar, b.q, b.A, b.B, b.Wc, s);
}

int vqhmm_regimes_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int64_t T, float* q,
                      int32_t* regimes, void* ws, size_t ws_bytes, void* stream) {
  if (!dims_ok(d) || !w || !x || !regimes || !ws || B < 0 || T < 0) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  size_t need;
  vqhmm_infer_workspace_size(d, B, T, &need);
  if (ws_bytes < need) return VQHMM_EWORKSPACE;
  InferBufs b = carve_infer(d, B, T, ws);
  return encode_impl(d, w, x, B, T, nullptr, q, nullptr, b.in, b.A, b.B, (hipStream_t)stream, regimes);
}

// ---------------------------------------------------------------- autograd of the module surface
// VAE_HMM.encode / decode / forward under autograd (VQ_VAE_HMM_fixed.py:100-104, :139-143): the module's forward
// recomputed into the workspace (ReLU outputs kept as the backward's masks), the data gradients on the conv
// kernels (transposed + flipped weights, ReLU-backward masks), the weight gradients as split-K slabs, and one
// fixed-order slab reduction (tail_kernel) into the flat gradient; the composed decoder conv1's dW / dE by
// compose_bwd.  Layers as ElboPlan::wl: 0 to_params, 1 dec_conv2, 2 dec_conv1 (composed), 3 to_logits,
// 4 enc_conv2, 5 enc_conv1.
namespace {
struct ModBwd {
  int64_t R;
  float *xin, *h1, *h2, *q, *dlog, *dh2, *dh1;
  float *qin, *g1, *g2, *dpar, *dg2, *dg1, *dq, *dqx, *zero, *Wc, *dWc;
  WLayer wl[6];
  size_t bytes;
};

ModBwd plan_modbwd(const vqhmm_dims_t* d, int64_t B, int64_t T, void* ws) {
  ModBwd m{};
  Carver c{reinterpret_cast<char*>(ws ? ws : reinterpret_cast<void*>(4096))};
  const int64_t R = B * (T + 2);
  const int D = d->input_dim, H = d->hidden_dim, H2 = d->hidden_dim2, K = d->K;
  m.R = R;
  m.xin = c.take<float>(R * ld4(D));
  m.h1 = c.take<float>(R * ld4(H));
  m.h2 = c.take<float>(R * ld4(H2));
  m.q = c.take<float>(R * ld4(K));
  m.dlog = c.take<float>(R * ld4(K));
  m.dh2 = c.take<float>(R * ld4(H2));
  m.dh1 = c.take<float>(R * ld4(H));
  m.qin = c.take<float>(R * ld4(K));
  m.g1 = c.take<float>(R * ld4(H));
  m.g2 = c.take<float>(R * ld4(H));
  m.dpar = c.take<float>(R * ld4(2 * D));
  m.dg2 = c.take<float>(R * ld4(H));
  m.dg1 = c.take<float>(R * ld4(H));
  m.dq = c.take<float>(R * ld4(K));
  m.dqx = c.take<float>(R * ld4(K));
  m.zero = c.take<float>(R * ld4(K));
  m.Wc = c.take<float>((size_t)H * K * 3);
  m.dWc = c.take<float>((size_t)H * K * 3);
  const int shapes[6][3] = {{2 * D, H, 1}, {H, H, 3}, {H, K, 3}, {K, H2, 1}, {H2, H, 3}, {H, D, 3}};
  for (int i = 0; i < 6; ++i) {
    WLayer& w = m.wl[i];
    w.N = shapes[i][0]; w.C = shapes[i][1]; w.ks = shapes[i][2];
    WgradArgs probe{};
    probe.N = w.N; probe.C = w.C; probe.ks = w.ks; probe.rows_per_chunk = 64;
    w.rows = (w.N <= 64 && w.C <= 64) ? wgrad2_rows(R, w.N, w.C, w.ks)
             : wgradbig_supported(probe) ? wgradbig_rows(R, w.N, w.C)
                                         : wgrad_chunks(R, cdiv(w.N, 64) * cdiv(w.C, 64));
    w.nchunks = cdiv(R, w.rows);
    w.slab = c.take<float>((size_t)w.nchunks * w.N * w.C * w.ks);
    w.bslab = c.take<float>((size_t)w.nchunks * w.N);
  }
  m.bytes = c.off + 256;
  return m;
}

ConvArgs mconv(const ModBwd& m, int T, const float* src, int Kc, int ks, const float* W, const float* bias, int N,
               int act, const float* aux, float* out, int w_dgrad) {
  ConvArgs a{};
  a.R = m.R; a.T = T;
  a.src = src; a.Kc = Kc; a.ks = ks; a.W = W; a.bias = bias; a.N = N; a.act = act; a.aux = aux; a.out = out;
  a.w_dgrad = w_dgrad;
  return a;
}

int mwgrad(const ModBwd& m, int T, int i, const float* dy, const float* x, hipStream_t s) {
  const WLayer& L = m.wl[i];
  WgradArgs wa{};
  wa.dy = dy; wa.x = x; wa.R = m.R; wa.T = T;
  wa.N = L.N; wa.C = L.C; wa.ks = L.ks; wa.rows_per_chunk = L.rows; wa.slab = L.slab; wa.bias_slab = L.bslab;
  return launch_wgrad(wa, s);
}

// encoder forward (x CF -> xin, h1, h2; with q_pcl: + to_logits and its softmax -> q_pcl)
int mod_enc_fwd(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int T, const ModBwd& m,
                float* q_pcl, hipStream_t s) {
  int rc;
  if ((rc = launch_to_pcl(x, d->input_dim, B, T, T, 1, m.xin, s))) return rc;
  if ((rc = launch_conv(mconv(m, T, m.xin, d->input_dim, 3, w[ENC1_W], w[ENC1_B], d->hidden_dim, 1, nullptr, m.h1, 0), s)))
    return rc;
  ConvArgs a = mconv(m, T, m.h1, d->hidden_dim, 3, w[ENC2_W], w[ENC2_B], d->hidden_dim2, 1, nullptr, m.h2, 0);
  if (q_pcl) {
    a.tW = w[LOGIT_W]; a.tb = w[LOGIT_B]; a.C2 = d->K; a.q_out = q_pcl;
  }
  return launch_conv(a, s);
}
// encoder backward from m.dlog: to_logits / enc_conv2 data gradients (+ enc_conv1's into dx, CF), weight gradients
int mod_enc_bwd(const vqhmm_dims_t* d, const float* const* w, int T, const ModBwd& m, float* dx, hipStream_t s) {
  int rc;
  if ((rc = launch_conv(mconv(m, T, m.dlog, d->K, 1, w[LOGIT_W], nullptr, d->hidden_dim2, 2, m.h2, m.dh2, 1), s)))
    return rc;
  if ((rc = launch_conv(mconv(m, T, m.dh2, d->hidden_dim2, 3, w[ENC2_W], nullptr, d->hidden_dim, 2, m.h1, m.dh1, 1), s)))
    return rc;
  if (dx) {
    ConvArgs a = mconv(m, T, m.dh1, d->hidden_dim, 3, w[ENC1_W], nullptr, d->input_dim, 0, nullptr, nullptr, 1);
    a.out_cf = dx;
    if ((rc = launch_conv(a, s))) return rc;
  }
  if ((rc = mwgrad(m, T, 3, m.dlog, m.h2, s))) return rc;
  if ((rc = mwgrad(m, T, 4, m.dh2, m.h1, s))) return rc;
  return mwgrad(m, T, 5, m.dh1, m.xin, s);
}
// decoder forward from q (PCL) -> g1, g2 (composed conv1 W' = W E^T into m.Wc)
int mod_dec_fwd(const vqhmm_dims_t* d, const float* const* w, const float* qp, int T, const ModBwd& m, hipStream_t s) {
  int rc;
  const int H = d->hidden_dim;
  if ((rc = launch_compose_fwd(w[DEC1_W], w[EMB], H, d->K, m.Wc, s))) return rc;
  if ((rc = launch_conv(mconv(m, T, qp, d->K, 3, m.Wc, w[DEC1_B], H, 1, nullptr, m.g1, 0), s))) return rc;
  return launch_conv(mconv(m, T, m.g1, H, 3, w[DEC2_W], w[DEC2_B], H, 1, nullptr, m.g2, 0), s);
}
// decoder backward from m.dpar: to_params / dec_conv2 / composed dec_conv1 data gradients (dq: PCL m.dq and/or CF
// dq_cf), weight gradients of the three layers
int mod_dec_bwd(const vqhmm_dims_t* d, const float* const* w, const float* qp, int T, const ModBwd& m, float* dq_cf,
                hipStream_t s) {
  int rc;
  const int H = d->hidden_dim;
  if ((rc = launch_conv(mconv(m, T, m.dpar, 2 * d->input_dim, 1, w[PAR_W], nullptr, H, 2, m.g2, m.dg2, 1), s))) return rc;
  if ((rc = launch_conv(mconv(m, T, m.dg2, H, 3, w[DEC2_W], nullptr, H, 2, m.g1, m.dg1, 1), s))) return rc;
  ConvArgs a = mconv(m, T, m.dg1, H, 3, m.Wc, nullptr, d->K, 0, nullptr, m.dq, 1);
  a.out_cf = dq_cf;
  if ((rc = launch_conv(a, s))) return rc;
  if ((rc = mwgrad(m, T, 0, m.dpar, m.g2, s))) return rc;
  if ((rc = mwgrad(m, T, 1, m.dg2, m.g1, s))) return rc;
  return mwgrad(m, T, 2, m.dg1, qp, s);
}
// the slabs of layers [i0, i1) summed into grad (the composed layer's dWc into m.dWc, then dW / dE)
int mod_reduce(const vqhmm_dims_t* d, const float* const* w, const ModBwd& m, int i0, int i1, float* g, hipStream_t s) {
  int64_t off[VQHMM_NPARAMS + 1];
  vqhmm_param_layout(d, off);
  const int wout[6] = {PAR_W, DEC2_W, DEC1_W, LOGIT_W, ENC2_W, ENC1_W};
  const int bout[6] = {PAR_B, DEC2_B, DEC1_B, LOGIT_B, ENC2_B, ENC1_B};
  TailArgs ta{};
  int n = 0;
  for (int i = i0; i < i1; ++i) {
    const WLayer& L = m.wl[i];
    float* wo = i == 2 ? m.dWc : g + off[wout[i]];
    ta.s[n++] = SlabSeg{L.slab, wo, nullptr, L.nchunks, (int64_t)L.N * L.C * L.ks, nullptr, 0, 0};
    ta.s[n++] = SlabSeg{L.bslab, g + off[bout[i]], nullptr, L.nchunks, L.N, nullptr, 0, 0};
  }
  ta.nseg = n;
  int rc;
  if ((rc = launch_grad_tail(ta, s))) return rc;
  if (i0 <= 2 && 2 < i1) {
    const LogPriorGradArgs lp{};
    return launch_compose_bwd(m.dWc, w[DEC1_W], w[EMB], d->hidden_dim, d->K, g + off[DEC1_W], g + off[EMB], lp, s);
  }
  return VQHMM_OK;
}
}  // namespace

int vqhmm_module_bwd_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* bytes) {
  if (!dims_ok(d) || B < 0 || T < 0 || !bytes) return VQHMM_EINVAL;
  *bytes = plan_modbwd(d, B, T, nullptr).bytes;
  return VQHMM_OK;
}

int vqhmm_encode_bwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const float* dlogits, int64_t B,
                         int64_t T, void* ws, size_t ws_bytes, float* grad, float* dx, void* stream) {
  if (!dims_ok(d) || !w || !x || !dlogits || !ws || !grad || B < 0 || T < 0) return VQHMM_EINVAL;
  for (int i = ENC1_W; i <= LOGIT_B; ++i)
    if (!w[i]) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  const ModBwd m = plan_modbwd(d, B, T, ws);
  if (ws_bytes < m.bytes) return VQHMM_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = mod_enc_fwd(d, w, x, B, (int)T, m, nullptr, s))) return rc;
  if ((rc = launch_to_pcl(dlogits, d->K, B, (int)T, T, 1, m.dlog, s))) return rc;
  if ((rc = mod_enc_bwd(d, w, (int)T, m, dx, s))) return rc;
  return mod_reduce(d, w, m, 3, 6, grad, s);
}

int vqhmm_decode_bwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* q, const float* dpar, int64_t B,
                         int64_t T, void* ws, size_t ws_bytes, float* grad, float* dq, void* stream) {
  if (!dims_ok(d) || !w || !q || !dpar || !ws || !grad || B < 0 || T < 0) return VQHMM_EINVAL;
  for (int i = EMB; i <= PAR_B; ++i)
    if (!w[i]) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  const ModBwd m = plan_modbwd(d, B, T, ws);
  if (ws_bytes < m.bytes) return VQHMM_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = launch_to_pcl(q, d->K, B, (int)T, T, 1, m.qin, s))) return rc;
  if ((rc = mod_dec_fwd(d, w, m.qin, (int)T, m, s))) return rc;
  if ((rc = launch_to_pcl(dpar, 2 * d->input_dim, B, (int)T, T, 1, m.dpar, s))) return rc;
  if ((rc = mod_dec_bwd(d, w, m.qin, (int)T, m, dq, s))) return rc;
  return mod_reduce(d, w, m, 0, 3, grad, s);
}

int vqhmm_forward_bwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const float* dpar,
                          const float* dq, int64_t B, int64_t T, void* ws, size_t ws_bytes, float* grad, float* dx,
                          void* stream) {
  if (!dims_ok(d) || !w || !x || !ws || !grad || B < 0 || T < 0) return VQHMM_EINVAL;
  for (int i = ENC1_W; i <= PAR_B; ++i)
    if (!w[i] && (i < LOG_PRIOR || i > TN2_B)) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  const ModBwd m = plan_modbwd(d, B, T, ws);
  if (ws_bytes < m.bytes) return VQHMM_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int Ti = (int)T;
  const size_t kbytes = (size_t)m.R * ld4(d->K) * sizeof(float);
  int rc;
  if ((rc = mod_enc_fwd(d, w, x, B, Ti, m, m.q, s))) return rc;  // q = softmax(logits) (PCL), the decoder's input
  if ((rc = mod_dec_fwd(d, w, m.q, Ti, m, s))) return rc;
  if (dpar) {
    if ((rc = launch_to_pcl(dpar, 2 * d->input_dim, B, Ti, T, 1, m.dpar, s))) return rc;
  } else if (hipMemsetAsync(m.dpar, 0, (size_t)m.R * ld4(2 * d->input_dim) * sizeof(float), s) != hipSuccess) {
    return VQHMM_ELAUNCH;
  }
  if ((rc = mod_dec_bwd(d, w, m.q, Ti, m, nullptr, s))) return rc;
  // dL/dq = the decoder's + the caller's (q is also an output); the softmax backward of q = softmax(logits)
  if (dq) {
    if ((rc = launch_to_pcl(dq, d->K, B, Ti, T, 1, m.dqx, s))) return rc;
  } else if (hipMemsetAsync(m.dqx, 0, kbytes, s) != hipSuccess) {
    return VQHMM_ELAUNCH;
  }
  if (hipMemsetAsync(m.zero, 0, kbytes, s) != hipSuccess) return VQHMM_ELAUNCH;
  if ((rc = launch_logits_bwd(m.q, m.dq, m.dqx, m.zero, nullptr, m.R, d->K, m.dlog, s))) return rc;
  if ((rc = mod_enc_bwd(d, w, Ti, m, dx, s))) return rc;
  return mod_reduce(d, w, m, 0, 6, grad, s);
}

int vqhmm_argmax_f32(const float* q, int64_t B, int64_t K, int64_t T, int32_t* idx, void* stream) {
  if (B < 0 || K < 1 || T < 0 || K > INT32_MAX || (B * T > 0 && (!q || !idx))) return VQHMM_EINVAL;
  return launch_argmax_cf(q, B, K, T, idx, (hipStream_t)stream);
}

int vqhmm_prior_f32(const vqhmm_dims_t* d, const float* const* w, const float* u, int u_layout, int64_t B, int64_t T,
                    float* log_pi, float* log_A, void* stream) {
  if (!dims_ok(d) || !w || !log_pi || !log_A || B < 0 || T < 0 || (B * T > 0 && !u)) return VQHMM_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = launch_log_softmax_vec(w[LOG_PRIOR], d->K, log_pi, s))) return rc;
  PriorArgs p{};
  p.B = B; p.T = (int)T; p.K = d->K; p.U = d->u_dim; p.TH = d->trans_hidden; p.u = u;
  if (u_layout == 0) { p.u_sc = T; p.u_st = 1; } else { p.u_sc = 1; p.u_st = d->u_dim; }
  p.W1 = w[TN0_W]; p.b1 = w[TN0_B]; p.W2 = w[TN2_W]; p.b2 = w[TN2_B]; p.log_A = log_A;
  return launch_prior_fwd(p, s);
}

// Autograd of Prior.forward alone (VQ_VAE_HMM_fixed.py:59-71): the MLP recomputed on PCL rows (1x1 convs), the
// log_softmax backward (prior_lsm_bwd), the hidden layer's masked data gradient and the two weight gradients,
// one slab reduction; du (CF (B, U, T), nullable) by the first layer's data gradient.
namespace {
struct PriorBwd {
  int64_t R;
  float *up, *hid, *lg, *dA, *dlg, *dhid;
  WLayer wl[2];  // 0: transition_net.2 (K^2, TH), 1: transition_net.0 (TH, U)
  size_t bytes;
};
PriorBwd plan_prior_bwd(const vqhmm_dims_t* d, int64_t B, int64_t T, void* ws) {
  PriorBwd p{};
  Carver c{reinterpret_cast<char*>(ws ? ws : reinterpret_cast<void*>(4096))};
  const int64_t R = B * (T + 2);
  const int K2 = d->K * d->K, TH = d->trans_hidden, U = d->u_dim;
  p.R = R;
  p.up = c.take<float>(R * ld4(U));
  p.hid = c.take<float>(R * ld4(TH));
  p.lg = c.take<float>(R * ld4(K2));
  p.dA = c.take<float>(R * ld4(K2));
  p.dlg = c.take<float>(R * ld4(K2));
  p.dhid = c.take<float>(R * ld4(TH));
  const int shapes[2][2] = {{K2, TH}, {TH, U}};
  for (int i = 0; i < 2; ++i) {
    WLayer& w = p.wl[i];
    w.N = shapes[i][0]; w.C = shapes[i][1]; w.ks = 1;
    WgradArgs probe{};
    probe.N = w.N; probe.C = w.C; probe.ks = 1; probe.rows_per_chunk = 64;
    w.rows = (w.N <= 64 && w.C <= 64) ? wgrad2_rows(R, w.N, w.C, 1)
             : wgradbig_supported(probe) ? wgradbig_rows(R, w.N, w.C)
                                         : wgrad_chunks(R, cdiv(w.N, 64) * cdiv(w.C, 64));
    w.nchunks = cdiv(R, w.rows);
    w.slab = c.take<float>((size_t)w.nchunks * w.N * w.C);
    w.bslab = c.take<float>((size_t)w.nchunks * w.N);
  }
  p.bytes = c.off + 256;
  return p;
}
}  // namespace

int vqhmm_prior_bwd_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* bytes) {
  if (!dims_ok(d) || B < 0 || T < 0 || !bytes) return VQHMM_EINVAL;
  *bytes = plan_prior_bwd(d, B, T, nullptr).bytes;
  return VQHMM_OK;
}

int vqhmm_prior_bwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* u, int u_layout,
                        const float* dlog_pi, const float* dlog_A, int64_t B, int64_t T, void* ws, size_t ws_bytes,
                        float* grad, float* du, void* stream) {
  if (!dims_ok(d) || !w || !ws || !grad || B < 0 || T < 0 || (B * T > 0 && (!u || !dlog_A))) return VQHMM_EINVAL;
  for (int i = LOG_PRIOR; i <= TN2_B; ++i)
    if (!w[i]) return VQHMM_EINVAL;
  const PriorBwd p = plan_prior_bwd(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  int64_t off[VQHMM_NPARAMS + 1];
  vqhmm_param_layout(d, off);
  hipStream_t s = (hipStream_t)stream;
  const int Ti = (int)T, K = d->K, K2 = K * K, TH = d->trans_hidden, U = d->u_dim;
  int rc;
  if (B * T == 0)  // only log_pi's gradient
    return launch_prior_lsm_bwd(nullptr, nullptr, 0, K, nullptr, w[LOG_PRIOR], dlog_pi, grad + off[LOG_PRIOR], s);
  ModBwd m{};  // mconv / mwgrad take the row count from it
  m.R = p.R;
  if ((rc = launch_to_pcl(u, U, B, Ti, u_layout == 0 ? T : 1, u_layout == 0 ? 1 : U, p.up, s))) return rc;
  if ((rc = launch_conv(mconv(m, Ti, p.up, U, 1, w[TN0_W], w[TN0_B], TH, 1, nullptr, p.hid, 0), s))) return rc;
  if ((rc = launch_conv(mconv(m, Ti, p.hid, TH, 1, w[TN2_W], w[TN2_B], K2, 0, nullptr, p.lg, 0), s))) return rc;
  if ((rc = launch_to_pcl(dlog_A, K2, B, Ti, 1, K2, p.dA, s))) return rc;  // (B, T, K, K) = (B, T, K^2)
  if ((rc = launch_prior_lsm_bwd(p.lg, p.dA, p.R, K, p.dlg, w[LOG_PRIOR], dlog_pi, grad + off[LOG_PRIOR], s))) return rc;
  if ((rc = launch_conv(mconv(m, Ti, p.dlg, K2, 1, w[TN2_W], nullptr, TH, 2, p.hid, p.dhid, 1), s))) return rc;
  if (du) {
    ConvArgs a = mconv(m, Ti, p.dhid, TH, 1, w[TN0_W], nullptr, U, 0, nullptr, nullptr, 1);
    a.out_cf = du;
    if ((rc = launch_conv(a, s))) return rc;
  }
  m.wl[0] = p.wl[0];
  m.wl[1] = p.wl[1];
  if ((rc = mwgrad(m, Ti, 0, p.dlg, p.hid, s))) return rc;
  if ((rc = mwgrad(m, Ti, 1, p.dhid, p.up, s))) return rc;
  TailArgs ta{};
  ta.s[0] = SlabSeg{p.wl[0].slab, grad + off[TN2_W], nullptr, p.wl[0].nchunks, (int64_t)K2 * TH, nullptr, 0, 0};
  ta.s[1] = SlabSeg{p.wl[0].bslab, grad + off[TN2_B], nullptr, p.wl[0].nchunks, K2, nullptr, 0, 0};
  ta.s[2] = SlabSeg{p.wl[1].slab, grad + off[TN0_W], nullptr, p.wl[1].nchunks, (int64_t)TH * U, nullptr, 0, 0};
  ta.s[3] = SlabSeg{p.wl[1].bslab, grad + off[TN0_B], nullptr, p.wl[1].nchunks, TH, nullptr, 0, 0};
  ta.nseg = 4;
  return launch_grad_tail(ta, s);
}

size_t vqhmm_prior_viterbi_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T) {
  if (!dims_ok(d) || B < 0 || T < 0) return 0;
  return 256 + viterbi_ws_bytes(B, T, d->K);
}

int vqhmm_prior_viterbi_f32(const vqhmm_dims_t* d, const float* const* w, const float* u, int u_layout,
                            const float* em, const int64_t* lengths, int64_t B, int64_t T, int32_t* path,
                            float* score, void* ws, size_t ws_bytes, void* stream) {
  if (!dims_ok(d) || !w || B < 0 || T < 0) return VQHMM_EINVAL;
  if (B == 0 || T == 0) return VQHMM_OK;
  if (!u || !em || !lengths || !path || !score) return VQHMM_EINVAL;
  PriorArgs p{};
  p.B = B; p.T = (int)T; p.K = d->K; p.U = d->u_dim; p.TH = d->trans_hidden; p.u = u;
  if (u_layout == 0) { p.u_sc = T; p.u_st = 1; } else { p.u_sc = 1; p.u_st = d->u_dim; }
  p.W1 = w[TN0_W]; p.b1 = w[TN0_B]; p.W2 = w[TN2_W]; p.b2 = w[TN2_B]; p.log_A = nullptr;
  if (!prior_viterbi_supported(p) || T > (1 << 28)) return VQHMM_EUNSUPPORTED;
  if (!ws || ws_bytes < vqhmm_prior_viterbi_workspace_size(d, B, T)) return VQHMM_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* log_pi = (float*)ws;
  int rc;
  if ((rc = launch_log_softmax_vec(w[LOG_PRIOR], d->K, log_pi, s))) return rc;
  return launch_prior_viterbi(p, log_pi, em, lengths, path, score, (char*)ws + 256, ws_bytes - 256, s);
}

}  // extern "C"
