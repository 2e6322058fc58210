"""Turn a tools/pmc.py result (per-kernel mean FETCH_SIZE / WRITE_SIZE per dispatch) into
profiles/pmc_traffic.json, the per-stage HBM traffic bench.py reports as roofline.traffic.

    python tools/make_pmc_traffic.py SRC.json [SRC2.json ...] profiles/pmc_traffic.json

Only stages that are ONE kernel launch (and whose kernel serves no other stage) are mapped.  Training-step
sections are keyed config/Bbatch (tools/gpu_pmc_all.sh profiles the default cfg2 batch, 1024): bench.py reports
a traffic figure only for the batch it was measured at.
FETCH_SIZE and WRITE_SIZE are rocprofv3 derived counters in KB; on gfx950 FETCH_SIZE counts half the
bytes of a wide streaming read, so HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(MI355X_MICROARCH.md, HBM section).
"""
import json
import sys

# (bench.py section, stage / kernel key) -> substring of the profiled kernel name
MAP = {
    ("cfg2/B1024", "elbo_head"): "elbo_head_pipe_kernel<3, 2, 8>",
    ("cfg2/B1024", "strip_fwd(enc_conv1+enc_conv2+to_logits+dec_conv1+dec_conv2+to_params)"): "strip_fwd_kernel<2, 0, 0>",
    ("cfg2/B1024", "to_params_dgrad+dec_conv2_dgrad"): "conv2f_kernel<4, 0, 1, 2, false, 1>",
    ("cfg2/B1024", "tail(slab reduction+composed dW/dE[+adam])"): "tail_kernel<true>",
    ("cfg2/B1024", "inputs_to_pcl+compose_fwd"): "prologue_kernel",
    ("cfg2/B1024", "wgrad_group(all 6 weight gradients)"): "wgrad2_group_kernel",
    ("cfg2/B1024", "dec_conv1_dgrad(+logits_bwd, to_logits_dgrad if K<=4)"): "conv2w_kernel<1, 4, 3, 3",
    ("cfg2/B1024", "enc_conv2_dgrad"): "conv2w_kernel<4, 2, 3, 2",
    ("vq_cfg3", "vq_argmin"): "vq_rows_kernel<16, 2, false, 2, false>",
    ("viterbi_cfg5", "viterbi_cfg5"): "viterbi_kernel<8, true>",
    ("fwdbwd_cfg4", "fwdbwd_cfg4"): "fwdbwd_kernel<8, true, true, 2>",
}


def main():
    srcs, dst = sys.argv[1:-1], sys.argv[-1]
    per_kernel = {}
    for src in srcs:
        per_kernel.update(json.load(open(src)))
    out = {}
    for (sec, key), sub in MAP.items():
        hits = [v for k, v in per_kernel.items() if sub in k]
        if len(hits) != 1 or "FETCH_SIZE" not in hits[0] or "WRITE_SIZE" not in hits[0]:
            continue
        h = hits[0]
        out.setdefault(sec, {})[key] = round(2 * h["FETCH_SIZE"] * 1024 + h["WRITE_SIZE"] * 1024)
    out["_note"] = ("HBM bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (rocprofv3 --pmc, separate passes, "
                    "gfx950 FETCH correction); sources " + ", ".join(srcs))
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
