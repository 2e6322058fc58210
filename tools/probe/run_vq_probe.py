"""VQ row-kernel ablation (tools/probe/libvqprobe.so) at cfg3: mode bit0 no next-tile loads,
bit1 no MFMA, bit2 no argmin epilogue."""
import ctypes
import json
import os
import sys

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvqprobe.so"))
B, Dv, T, K = 2048, 64, 200, 32
g = torch.Generator(device="cuda").manual_seed(1)
z = torch.randn(B, Dv, T, device="cuda", generator=g)
cb = torch.randn(K, Dv, device="cuda", generator=g)
idx = torch.empty(B, T, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
wpcs = [int(w) for w in sys.argv[1:]] or [8]
for wpc in wpcs:
    for mode in range(8):
        run = lambda: lib.vq_probe(mode, ctypes.c_void_p(z.data_ptr()), B, Dv, T, ctypes.c_void_p(cb.data_ptr()), K,
                                   ctypes.c_void_p(idx.data_ptr()), wpc, ctypes.c_void_p(st.cuda_stream))
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        print(json.dumps({"wpc": wpc, "mode": mode, "us": round(e0.elapsed_time(e1) / 20 * 1e3, 2)}), flush=True)
