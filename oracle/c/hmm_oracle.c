/* C restatement of the bit-exact integer-output kernels — TEST INFRASTRUCTURE.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (oracle/_build/liboracle.so); the product never links it.
 *
 * Contracts: see oracle/hmm_ref.py (module docstring).  Semantic sources:
 *   VQ argmin  pseudocode.txt:11-18, backtesting.py:154-155 (reference)
 *   Viterbi    math.md:23-67; tables of Prior.forward VQ_VAE_HMM_fixed.py:59-71,
 *              t-1 -> t indexing of log_A as in :125-127.
 * Built with -ffp-contract=off: the only fused multiply-adds are the explicit
 * fmaf() chains of the VQ score, which the GPU kernel mirrors (its f32 MFMA is
 * bit-for-bit a k-ordered fmaf chain).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* z: (B, Dv, T) channels-first, codebook: (K, Dv). idx/dmin: (B, T).
 * Expansion-form contract (see oracle/hmm_ref.py):
 *   cn_k  = fmaf chain over d of c[k,d]*c[k,d] from +0
 *   s_k   = fmaf chain over d of z[d]*(-2 c[k,d]) starting from cn_k
 *   idx   = first k with the smallest s_k
 *   dmin  = s_idx + ((q0 + q1) + (q2 + q3)), q_r = fmaf chain of z[d]^2 over d = r (mod 4) */
void oracle_vq_argmin_f32(const float* z, int64_t B, int64_t Dv, int64_t T,
                          const float* cb, int64_t K, int32_t* idx, float* dmin) {
    float* zz = (float*)malloc(sizeof(float) * (size_t)(Dv > 0 ? Dv : 1));
    float* cn = (float*)malloc(sizeof(float) * (size_t)(K > 0 ? K : 1));
    for (int64_t k = 0; k < K; ++k) {
        float acc = 0.0f;
        for (int64_t d = 0; d < Dv; ++d) acc = fmaf(cb[k * Dv + d], cb[k * Dv + d], acc);
        cn[k] = acc;
    }
    for (int64_t b = 0; b < B; ++b) {
        for (int64_t t = 0; t < T; ++t) {
            float q[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int64_t d = 0; d < Dv; ++d) {
                zz[d] = z[(b * Dv + d) * T + t];
                q[d & 3] = fmaf(zz[d], zz[d], q[d & 3]);
            }
            float best = INFINITY;
            int32_t arg = 0;
            for (int64_t k = 0; k < K; ++k) {
                float acc = cn[k];
                const float* c = cb + k * Dv;
                for (int64_t d = 0; d < Dv; ++d) acc = fmaf(zz[d], -2.0f * c[d], acc);
                if (acc < best) { best = acc; arg = (int32_t)k; }
            }
            idx[b * T + t] = arg;
            if (dmin) dmin[b * T + t] = best + ((q[0] + q[1]) + (q[2] + q[3]));
        }
    }
    free(cn);
    free(zz);
}

/* log_pi (K), log_A (B,T,K,K), em (B,T,K), lengths (B) -> path (B,T), score (B). */
void oracle_viterbi_f32(const float* log_pi, const float* log_A, const float* em,
                        const int64_t* lengths, int64_t B, int64_t T, int64_t K,
                        int32_t* path, float* score) {
    float* delta = (float*)malloc(sizeof(float) * (size_t)K);
    float* nd = (float*)malloc(sizeof(float) * (size_t)K);
    int32_t* bp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(T > 0 ? T : 1) * (size_t)K);  /* any K */
    for (int64_t b = 0; b < B; ++b) {
        int64_t L = lengths[b] < T ? lengths[b] : T;
        for (int64_t t = 0; t < T; ++t) path[b * T + t] = -1;
        if (L <= 0) { score[b] = -INFINITY; continue; }
        const float* e = em + b * T * K;
        const float* A = log_A + b * T * K * K;
        for (int64_t j = 0; j < K; ++j) delta[j] = log_pi[j] + e[j];
        for (int64_t t = 1; t < L; ++t) {
            const float* At = A + t * K * K;
            for (int64_t j = 0; j < K; ++j) {
                float best = delta[0] + At[j];
                int arg = 0;
                for (int64_t i = 1; i < K; ++i) {
                    float v = delta[i] + At[i * K + j];
                    if (v > best) { best = v; arg = (int)i; }
                }
                nd[j] = best + e[t * K + j];
                bp[t * K + j] = arg;
            }
            memcpy(delta, nd, sizeof(float) * (size_t)K);
        }
        int64_t s = 0;
        for (int64_t j = 1; j < K; ++j) if (delta[j] > delta[s]) s = j;
        score[b] = delta[s];
        path[b * T + L - 1] = (int32_t)s;
        for (int64_t t = L - 1; t > 0; --t) {
            s = bp[t * K + s];
            path[b * T + t - 1] = (int32_t)s;
        }
    }
    free(delta); free(nd); free(bp);
}
