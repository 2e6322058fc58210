"""conv2 ablation (tools/probe/libconv2probe.so) at the cfg2 dec_conv2+to_params shape
(R = 1024*202 rows, 64 -> 64 channels, k=3, ReLU, tail 10): mode bit0 no MFMA, bit1 no epilogue,
bit2 no X staging."""
import ctypes
import json
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libconv2probe.so"))
B, T = 1024, 200
R = B * (T + 2)
g = torch.Generator(device="cuda").manual_seed(1)
src = torch.randn(R, 64, device="cuda", generator=g)
W = torch.randn(64, 64, 3, device="cuda", generator=g) * 0.1
bias = torch.randn(64, device="cuda", generator=g)
tW = torch.randn(10, 64, device="cuda", generator=g)
tb = torch.randn(10, device="cuda", generator=g)
out = torch.empty(R, 64, device="cuda")
t_out = torch.empty(R, 12, device="cuda")
st = torch.cuda.current_stream()
P = lambda t: ctypes.c_void_p(t.data_ptr())
flops = 2.0 * B * T * 64 * 64 * 3
for mode in range(8):
    run = lambda: lib.conv2_probe(mode, P(src), P(W), P(bias), P(tW), P(tb), 10, ctypes.c_int64(R), T, P(out),
                                  P(t_out), ctypes.c_void_p(st.cuda_stream))
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(20):
        run()
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(json.dumps({"mode": mode, "us": round(us, 2), "TFLOPs_if_full": round(flops / us / 1e6, 1)}), flush=True)
