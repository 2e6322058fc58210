"""Forward-backward launch time vs T at a fixed batch (slope = per-step chain cost, intercept = fixed
cost: ramp-up + gamma pass).   usage: python tools/fb_probe.py [B] [K]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd"))


def main():
    import vqhmm
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    g = torch.Generator(device="cuda").manual_seed(0)
    for T in (64, 128, 256, 512, 1024):
        log_pi = torch.log_softmax(torch.randn(K, device="cuda", generator=g), -1)
        log_A = torch.log_softmax(1.5 * torch.randn(B, T, K, K, device="cuda", generator=g), -1)
        em = torch.log_softmax(2.0 * torch.randn(B, T, K, device="cuda", generator=g), -1)
        for _ in range(3):
            vqhmm.forward_backward(log_pi, log_A, em)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            vqhmm.forward_backward(log_pi, log_A, em)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        print(f"B={B} K={K} T={T:5d}: {us:8.1f} us/call (incl. allocations)  {us / T * 1e3:7.1f} ns/step")


if __name__ == "__main__":
    main()
