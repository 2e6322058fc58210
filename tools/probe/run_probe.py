"""f32 MFMA throughput calibration (tools/probe/libprobe.so): TFLOP/s per (shape, chains, waves/SIMD)."""
import ctypes
import json
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe.so"))
out = torch.empty(1024 * 256 * 4, device="cuda")
st = torch.cuda.current_stream()
for shape, flops in ((32, 32 * 32 * 2 * 2), (16, 16 * 16 * 4 * 2)):
    for ch in ((1, 2, 4) if shape == 32 else (1, 2, 4, 8)):
        for wps in (1, 2, 4):
            blocks, iters = 256 * wps, 2000
            run = lambda: lib.probe(shape, ch, blocks, iters, ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(st.cuda_stream))
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 5 * 1e-3
            tf = blocks * 4 * iters * ch * flops / t / 1e12
            print(json.dumps({"shape": shape, "chains": ch, "waves_per_simd": wps, "us": round(t * 1e6, 1),
                              "TFLOPs": round(tf, 1)}), flush=True)
