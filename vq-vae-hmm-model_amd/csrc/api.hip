// extern "C" entry points of libvqhmm.so (declared in include/vqhmm.h).
#include "vqhmm.h"

#include "common.h"

namespace vqhmm {
int launch_vq_argmin(const float* z, int64_t B, int64_t Dv, int64_t T, const float* cb, int64_t K,
                     int32_t* idx, float* dmin, hipStream_t s);
}  // namespace vqhmm

using namespace vqhmm;

extern "C" {

int32_t vqhmm_abi_version(void) { return 1; }

int vqhmm_param_layout(const vqhmm_dims_t* d, int64_t off[VQHMM_NPARAMS + 1]) {
  if (!d || !off) return VQHMM_EINVAL;
  const int64_t D = d->input_dim, H = d->hidden_dim, K = d->K, H2 = d->hidden_dim2, U = d->u_dim,
                TH = d->trans_hidden;
  if (D <= 0 || H <= 0 || K <= 0 || H2 <= 0 || U <= 0 || TH <= 0) return VQHMM_EINVAL;
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

}  // extern "C"
