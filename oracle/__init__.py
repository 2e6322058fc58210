"""CPU oracle for the VAE_HMM hot path — TEST INFRASTRUCTURE ONLY.

Nothing in the product package (`vq-vae-hmm-model_amd/vqhmm`) imports this
package.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may use it, and only as the checker / the timed CPU
baseline, never as the thing measured or shipped.

Contents
  ref_model.py  torch-CPU restatement of the reference model + train loop
                (VQ_VAE_HMM_fixed.py:31-179), pinned bit-for-bit against the
                golden fixtures captured from the reference in tests/golden/.
  hmm_ref.py    numpy restatement of the three kernels the reference only
                specifies in prose (VQ argmin, HMM forward-backward, Viterbi),
                pinned by brute-force known-answer tests (tests/test_oracle_hmm.py).
  c/            C restatement of the bit-exact integer-output kernels
                (VQ argmin with an fmaf chain, fp32 max-plus Viterbi) for
                large-size checks and the timed CPU baseline.
"""
