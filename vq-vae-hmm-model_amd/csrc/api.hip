// extern "C" entry points of libvqhmm.so (declared in include/vqhmm.h) and the
// native executor of the VAE_HMM training step: it plans the workspace and
// enqueues the forward (5 kernels + finalize) and backward (~16 kernels)
// passes on the caller's stream.  See DESIGN.md for the kernel list.
#include "vqhmm.h"

#include <math.h>

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
};

struct ElboPlan {
  int64_t B, R;
  int T, D, H, H2, K, U, TH;
  int hgrid;
  // forward
  float *h1e, *h2e, *logits, *q, *g1, *g2, *par, *Wc;
  // head
  float *dpar, *dqx, *dlx;
  double* part;
  float *sW1, *sb1, *sW2, *sb2, *sq0;
  float *loss, *pieces;
  // backward
  float *dg2, *dg1, *dqd, *dlog, *dh2, *dh1, *dWc, *q0sum;
  WLayer wl[6];  // 0 to_params, 1 dec2, 2 dec1', 3 to_logits, 4 enc2, 5 enc1
  size_t bytes;
};

ElboPlan plan_elbo(const vqhmm_dims_t* d, int64_t B, int64_t T, void* ws) {
  ElboPlan p{};
  p.B = B; p.T = (int)T; p.R = B * (T + 2);
  p.D = d->input_dim; p.H = d->hidden_dim; p.H2 = d->hidden_dim2; p.K = d->K; p.U = d->u_dim; p.TH = d->trans_hidden;
  const int64_t R = p.R;
  const int H = p.H, H2 = p.H2, K = p.K, D = p.D;
  Carver c{reinterpret_cast<char*>(ws)};
  p.h1e = c.take<float>(R * H);
  p.h2e = c.take<float>(R * H2);
  p.logits = c.take<float>(R * K);
  p.q = c.take<float>(R * K);
  p.g1 = c.take<float>(R * H);
  p.g2 = c.take<float>(R * H);
  p.par = c.take<float>(R * 2 * D);
  p.Wc = c.take<float>((size_t)H * K * 3);
  p.hgrid = head_grid(R);
  p.dpar = c.take<float>(R * 2 * D);
  p.dqx = c.take<float>(R * K);
  p.dlx = c.take<float>(R * K);
  p.part = c.take<double>((size_t)p.hgrid * 4);
  p.sW1 = c.take<float>((size_t)p.hgrid * p.TH * p.U);
  p.sb1 = c.take<float>((size_t)p.hgrid * p.TH);
  p.sW2 = c.take<float>((size_t)p.hgrid * K * K * p.TH);
  p.sb2 = c.take<float>((size_t)p.hgrid * K * K);
  p.sq0 = c.take<float>((size_t)p.hgrid * K);
  p.loss = c.take<float>(1);
  p.pieces = c.take<float>(4);
  p.dg2 = c.take<float>(R * H);
  p.dg1 = c.take<float>(R * H);
  p.dqd = c.take<float>(R * K);
  p.dlog = c.take<float>(R * K);
  p.dh2 = c.take<float>(R * H2);
  p.dh1 = c.take<float>(R * H);
  p.dWc = c.take<float>((size_t)H * K * 3);
  p.q0sum = c.take<float>(K);
  const int shapes[6][3] = {{2 * D, H, 1}, {H, H, 3}, {H, K, 3}, {K, H2, 1}, {H2, H, 3}, {H, D, 3}};
  for (int i = 0; i < 6; ++i) {
    WLayer& w = p.wl[i];
    w.N = shapes[i][0]; w.C = shapes[i][1]; w.ks = shapes[i][2];
    const int64_t tiles = cdiv(w.N, 64) * cdiv(w.C, 64);
    w.rows = wgrad_chunks(R, tiles);
    w.nchunks = cdiv(R, w.rows);
    w.slab = c.take<float>((size_t)w.nchunks * w.N * w.C * w.ks);
    w.bslab = c.take<float>((size_t)w.nchunks * w.N);
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

int32_t vqhmm_abi_version(void) { return 1; }

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

int vqhmm_elbo_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* bytes) {
  if (!dims_ok(d) || B < 0 || T < 0 || !bytes) return VQHMM_EINVAL;
  *bytes = plan_elbo(d, B, T, nullptr).bytes;
  return VQHMM_OK;
}

int vqhmm_elbo_fwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, const float* u, int u_layout,
                       const int64_t* lengths, int64_t B, int64_t T, float beta, int need_grad, void* ws,
                       size_t ws_bytes, float* loss, double* loss_accum, void* stream) {
  if (!dims_ok(d) || !w || B <= 0 || T <= 0 || !x || !u || !lengths || !ws || !loss) return VQHMM_EINVAL;
  for (int i = 0; i < VQHMM_NPARAMS; ++i)
    if (!w[i]) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  // F0: composed decoder conv1 weight
  if ((rc = launch_compose_fwd(w[DEC1_W], w[EMB], p.H, p.K, p.Wc, s))) return rc;
  // F1: encoder.conv1 + ReLU, x read channels-first
  ConvArgs a = conv_base(p);
  a.src = x; a.src_cf = 1; a.Kc = p.D; a.ks = 3; a.W = w[ENC1_W]; a.bias = w[ENC1_B]; a.N = p.H; a.act = 1;
  a.out = p.h1e;
  if ((rc = launch_conv(a, s))) return rc;
  // F2: encoder.conv2 + ReLU, fused to_logits tail + softmax -> logits, q
  a = conv_base(p);
  a.src = p.h1e; a.Kc = p.H; a.ks = 3; a.W = w[ENC2_W]; a.bias = w[ENC2_B]; a.N = p.H2; a.act = 1; a.out = p.h2e;
  a.tW = w[LOGIT_W]; a.tb = w[LOGIT_B]; a.C2 = p.K; a.t_out = p.logits; a.q_out = p.q;
  if ((rc = launch_conv(a, s))) return rc;
  // F3: decoder.conv1 on q with the composed weight + ReLU
  a = conv_base(p);
  a.src = p.q; a.Kc = p.K; a.ks = 3; a.W = p.Wc; a.bias = w[DEC1_B]; a.N = p.H; a.act = 1; a.out = p.g1;
  if ((rc = launch_conv(a, s))) return rc;
  // F4: decoder.conv2 + ReLU, fused to_params tail -> (mu | logvar)
  a = conv_base(p);
  a.src = p.g1; a.Kc = p.H; a.ks = 3; a.W = w[DEC2_W]; a.bias = w[DEC2_B]; a.N = p.H; a.act = 1; a.out = p.g2;
  a.tW = w[PAR_W]; a.tb = w[PAR_B]; a.C2 = 2 * p.D; a.t_out = p.par;
  if ((rc = launch_conv(a, s))) return rc;
  // F5: fused ELBO head (+ its gradients when need_grad)
  HeadArgs h{};
  h.B = B; h.T = p.T; h.R = p.R; h.D = p.D; h.K = p.K; h.U = p.U; h.TH = p.TH;
  h.x = x; h.u = u;
  if (u_layout == 0) { h.u_sc = T; h.u_st = 1; } else { h.u_sc = 1; h.u_st = p.U; }
  h.lengths = lengths; h.par = p.par; h.logits = p.logits; h.q = p.q;
  h.W1 = w[TN0_W]; h.b1 = w[TN0_B]; h.W2 = w[TN2_W]; h.b2 = w[TN2_B]; h.log_prior = w[LOG_PRIOR];
  h.beta = beta; h.need_grad = need_grad;
  h.dpar = p.dpar; h.dqx = p.dqx; h.dlx = p.dlx; h.part = p.part;
  h.slab_W1 = p.sW1; h.slab_b1 = p.sb1; h.slab_W2 = p.sW2; h.slab_b2 = p.sb2; h.slab_q0 = p.sq0;
  if ((rc = launch_head(h, p.hgrid, s))) return rc;
  return launch_finalize_loss(p.part, p.hgrid, lengths, B, p.T, p.D, beta, loss, loss_accum, p.pieces, s);
}

int vqhmm_elbo_bwd_f32(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int64_t T,
                       float beta, const float* grad_scale, void* ws, size_t ws_bytes, float* g, void* stream) {
  if (!dims_ok(d) || !w || B <= 0 || T <= 0 || !x || !ws || !g) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, ws);
  if (ws_bytes < p.bytes) return VQHMM_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int64_t off[VQHMM_NPARAMS + 1];
  vqhmm_param_layout(d, off);
  int rc;
  // B1: to_params data grad (1x1, transposed) * ReLU'(g2), scaled by grad_scale
  ConvArgs a = conv_base(p);
  a.src = p.dpar; a.Kc = 2 * p.D; a.ks = 1; a.W = w[PAR_W]; a.w_dgrad = 1; a.scale = grad_scale; a.N = p.H;
  a.act = 2; a.aux = p.g2; a.out = p.dg2;
  if ((rc = launch_conv(a, s))) return rc;
  // B2: decoder.conv2 data grad * ReLU'(g1)
  a = conv_base(p);
  a.src = p.dg2; a.Kc = p.H; a.ks = 3; a.W = w[DEC2_W]; a.w_dgrad = 1; a.N = p.H; a.act = 2; a.aux = p.g1;
  a.out = p.dg1;
  if ((rc = launch_conv(a, s))) return rc;
  // B3: composed decoder.conv1 data grad -> dq (decoder path)
  a = conv_base(p);
  a.src = p.dg1; a.Kc = p.H; a.ks = 3; a.W = p.Wc; a.w_dgrad = 1; a.N = p.K; a.act = 0; a.out = p.dqd;
  if ((rc = launch_conv(a, s))) return rc;
  // B4: softmax backward (+ prior and entropy terms) -> dlogits
  if ((rc = launch_logits_bwd(p.q, p.dqd, p.dqx, p.dlx, grad_scale, p.R, p.K, p.dlog, s))) return rc;
  // B5: to_logits data grad * ReLU'(h2e)
  a = conv_base(p);
  a.src = p.dlog; a.Kc = p.K; a.ks = 1; a.W = w[LOGIT_W]; a.w_dgrad = 1; a.N = p.H2; a.act = 2; a.aux = p.h2e;
  a.out = p.dh2;
  if ((rc = launch_conv(a, s))) return rc;
  // B6: encoder.conv2 data grad * ReLU'(h1e)
  a = conv_base(p);
  a.src = p.dh2; a.Kc = p.H2; a.ks = 3; a.W = w[ENC2_W]; a.w_dgrad = 1; a.N = p.H; a.act = 2; a.aux = p.h1e;
  a.out = p.dh1;
  if ((rc = launch_conv(a, s))) return rc;
  // weight gradients (split-K partial slabs)
  const float* dys[6] = {p.dpar, p.dg2, p.dg1, p.dlog, p.dh2, p.dh1};
  const float* xs[6] = {p.g2, p.g1, p.q, p.h2e, p.h1e, x};
  for (int i = 0; i < 6; ++i) {
    const WLayer& L = p.wl[i];
    WgradArgs wa{};
    wa.dy = dys[i]; wa.x = xs[i]; wa.x_cf = (i == 5); wa.R = p.R; wa.T = p.T;
    wa.N = L.N; wa.C = L.C; wa.ks = L.ks; wa.rows_per_chunk = L.rows; wa.slab = L.slab; wa.bias_slab = L.bslab;
    if ((rc = launch_wgrad(wa, s))) return rc;
  }
  // reduce every slab into the flat gradient (fixed order)
  SlabSeg segs[18];
  int n = 0;
  auto seg = [&](const float* slab, int64_t nch, int64_t len, float* out, const float* scale) {
    segs[n++] = SlabSeg{slab, out, scale, nch, len};
  };
  const WLayer* wl = p.wl;
  seg(wl[0].slab, wl[0].nchunks, (int64_t)wl[0].N * wl[0].C, g + off[PAR_W], grad_scale);  // dpar is unscaled
  seg(wl[0].bslab, wl[0].nchunks, wl[0].N, g + off[PAR_B], grad_scale);
  seg(wl[1].slab, wl[1].nchunks, (int64_t)wl[1].N * wl[1].C * 3, g + off[DEC2_W], nullptr);
  seg(wl[1].bslab, wl[1].nchunks, wl[1].N, g + off[DEC2_B], nullptr);
  seg(wl[2].slab, wl[2].nchunks, (int64_t)wl[2].N * wl[2].C * 3, p.dWc, nullptr);
  seg(wl[2].bslab, wl[2].nchunks, wl[2].N, g + off[DEC1_B], nullptr);
  seg(wl[3].slab, wl[3].nchunks, (int64_t)wl[3].N * wl[3].C, g + off[LOGIT_W], nullptr);
  seg(wl[3].bslab, wl[3].nchunks, wl[3].N, g + off[LOGIT_B], nullptr);
  seg(wl[4].slab, wl[4].nchunks, (int64_t)wl[4].N * wl[4].C * 3, g + off[ENC2_W], nullptr);
  seg(wl[4].bslab, wl[4].nchunks, wl[4].N, g + off[ENC2_B], nullptr);
  seg(wl[5].slab, wl[5].nchunks, (int64_t)wl[5].N * wl[5].C * 3, g + off[ENC1_W], nullptr);
  seg(wl[5].bslab, wl[5].nchunks, wl[5].N, g + off[ENC1_B], nullptr);
  seg(p.sW1, p.hgrid, (int64_t)p.TH * p.U, g + off[TN0_W], grad_scale);
  seg(p.sb1, p.hgrid, p.TH, g + off[TN0_B], grad_scale);
  seg(p.sW2, p.hgrid, (int64_t)p.K * p.K * p.TH, g + off[TN2_W], grad_scale);
  seg(p.sb2, p.hgrid, (int64_t)p.K * p.K, g + off[TN2_B], grad_scale);
  seg(p.sq0, p.hgrid, p.K, p.q0sum, nullptr);
  if ((rc = launch_reduce_slabs(segs, n, s))) return rc;
  if ((rc = launch_compose_bwd(p.dWc, w[DEC1_W], w[EMB], p.H, p.K, g + off[DEC1_W], g + off[EMB], s))) return rc;
  return launch_log_prior_grad(p.q0sum, w[LOG_PRIOR], p.K, -beta / (float)B, grad_scale, g + off[LOG_PRIOR], s);
}

int vqhmm_elbo_pieces(const vqhmm_dims_t* d, int64_t B, int64_t T, const void* ws, const float** loss,
                      const float** pieces) {
  if (!dims_ok(d) || !ws) return VQHMM_EINVAL;
  ElboPlan p = plan_elbo(d, B, T, const_cast<void*>(ws));
  if (loss) *loss = p.loss;
  if (pieces) *pieces = p.pieces;
  return VQHMM_OK;
}

int vqhmm_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                   double beta1, double beta2, double eps, int64_t* step, float grad_scale, void* stream) {
  if (n < 0 || !step || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq))) return VQHMM_EINVAL;
  return launch_adam(param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, step, grad_scale,
                     (hipStream_t)stream);
}

// ---------------------------------------------------------------- inference surface
int vqhmm_infer_workspace_size(const vqhmm_dims_t* d, int64_t B, int64_t T, size_t* bytes) {
  if (!dims_ok(d) || B < 0 || T < 0 || !bytes) return VQHMM_EINVAL;
  const int64_t R = B * (T + 2);
  Carver c{nullptr};
  c.take<float>(R * d->hidden_dim);
  c.take<float>(R * d->hidden_dim);
  c.take<float>(R * d->K);
  c.take<float>((size_t)d->hidden_dim * d->K * 3);
  *bytes = c.off + 256;
  return VQHMM_OK;
}

static int encode_impl(const vqhmm_dims_t* d, const float* const* w, const float* x, int64_t B, int64_t T,
                       float* logits_cf, float* q_cf, float* q_pcl, float* bufA, float* bufB, hipStream_t s) {
  const int64_t R = B * (T + 2);
  ConvArgs a{};
  a.R = R; a.T = (int)T;
  a.src = x; a.src_cf = 1; a.Kc = d->input_dim; a.ks = 3; a.W = w[ENC1_W]; a.bias = w[ENC1_B];
  a.N = d->hidden_dim; a.act = 1; a.out = bufA;
  int rc;
  if ((rc = launch_conv(a, s))) return rc;
  a = ConvArgs{};
  a.R = R; a.T = (int)T;
  a.src = bufA; a.Kc = d->hidden_dim; a.ks = 3; a.W = w[ENC2_W]; a.bias = w[ENC2_B]; a.N = d->hidden_dim2;
  a.act = 1; a.out = bufB;
  a.tW = w[LOGIT_W]; a.tb = w[LOGIT_B]; a.C2 = d->K;
  if (logits_cf) { a.t_cf0 = logits_cf; a.t_split = d->K; }
  a.q_out = q_pcl;
  a.q_cf = q_cf;
  if (logits_cf && q_cf) return VQHMM_EINVAL;
  return launch_conv(a, s);
}

static int decode_impl(const vqhmm_dims_t* d, const float* const* w, const float* q, int q_cf, int64_t B,
                       int64_t T, float* mu, float* logvar, float* bufA, float* bufB, float* Wc, hipStream_t s) {
  const int64_t R = B * (T + 2);
  int rc;
  if ((rc = launch_compose_fwd(w[DEC1_W], w[EMB], d->hidden_dim, d->K, Wc, s))) return rc;
  ConvArgs a{};
  a.R = R; a.T = (int)T;
  a.src = q; a.src_cf = q_cf; a.Kc = d->K; a.ks = 3; a.W = Wc; a.bias = w[DEC1_B]; a.N = d->hidden_dim;
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

struct InferBufs { float *A, *B, *q, *Wc; };
static InferBufs carve_infer(const vqhmm_dims_t* d, int64_t B, int64_t T, void* ws) {
  const int64_t R = B * (T + 2);
  Carver c{reinterpret_cast<char*>(ws)};
  InferBufs b;
  b.A = c.take<float>(R * d->hidden_dim);
  b.B = c.take<float>(R * d->hidden_dim);
  b.q = c.take<float>(R * d->K);
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
  return encode_impl(d, w, x, B, T, logits, nullptr, nullptr, b.A, b.B, (hipStream_t)stream);
}

int vqhmm_decode_f32(const vqhmm_dims_t* d, const float* const* w, const float* q, int64_t B, int64_t T, float* mu,
                     float* logvar, void* ws, size_t ws_bytes, void* stream) {
  if (!dims_ok(d) || !w || !q || !mu || !logvar || !ws || B < 0 || T < 0) return VQHMM_EINVAL;
  if (B * T == 0) return VQHMM_OK;
  size_t need;
  vqhmm_infer_workspace_size(d, B, T, &need);
  if (ws_bytes < need) return VQHMM_EWORKSPACE;
  InferBufs b = carve_infer(d, B, T, ws);
  return decode_impl(d, w, q, 1, B, T, mu, logvar, b.A, b.B, b.Wc, (hipStream_t)stream);
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
  if ((rc = encode_impl(d, w, x, B, T, nullptr, q, b.q, b.A, b.B, s))) return rc;
  return decode_impl(d, w, b.q, 0, B, T, mu, logvar, b.A, b.B, b.Wc, s);
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

}  // extern "C"
