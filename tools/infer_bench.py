"""End-to-end viterbi_regimes cost split: encoder + emission
log_softmax, Prior.forward (log_A materialised), Viterbi, vs the fused Prior-MLP -> Viterbi
kernel (vqhmm_prior_viterbi_f32), at a cfg5-shaped shard.
usage: python tools/infer_bench.py [B] [T]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd"))


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        out = fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3, out


def main():
    import vqhmm
    from vqhmm.hmm import viterbi
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    K, D, H, H2, U, TH = 8, 16, 64, 32, 4, 128
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH).cuda()
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, D, T, device="cuda", generator=g)
    u = torch.randn(B, U, T, device="cuda", generator=g)
    with torch.no_grad():
        t_enc, em = timeit(lambda: torch.log_softmax(m.encode(x), dim=1).transpose(1, 2).contiguous())
        t_pri, (log_pi, log_A) = timeit(lambda: m.prior(u))
        t_vit, ref = timeit(lambda: viterbi(log_pi, log_A, em, None))
        t_fus, got = timeit(lambda: vqhmm.prior_viterbi(m.prior, u, em))
        t_all0, _ = timeit(lambda: vqhmm.viterbi_regimes(m, x, u, fused=False))
        t_all, _ = timeit(lambda: vqhmm.viterbi_regimes(m, x, u))
    gb = log_A.numel() * 4 / 1e9
    print(f"B={B} T={T} K={K}: encode+log_softmax {t_enc:.0f} us, prior (log_A {gb:.2f} GB) {t_pri:.0f} us, "
          f"viterbi {t_vit:.0f} us | fused prior+viterbi {t_fus:.0f} us (identical paths) | "
          f"viterbi_regimes end-to-end unfused {t_all0:.0f} us, fused {t_all:.0f} us")
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), "fused path differs"


if __name__ == "__main__":
    main()
