"""Turn a tools/pmc.py result (per-kernel mean FETCH_SIZE / WRITE_SIZE per dispatch) into
profiles/pmc_traffic.json, the per-stage HBM traffic bench.py reports as roofline.traffic.

    python tools/make_pmc_traffic.py cfg2/B1024=STEP.json [cfg2/B128=STEP128.json ...] LEG.json [...] profiles/pmc_traffic.json

Only stages that are ONE kernel launch (and whose kernel serves no other stage) are mapped.  Training-step
sources are given as SECTION=path, the section keyed config/Bbatch (tools/gpu_pmc_all.sh profiles cfg2 at
1024 and at the B = 128 shard): bench.py reports a traffic figure only for the batch it was measured at.
FETCH_SIZE and WRITE_SIZE are rocprofv3 derived counters in KB; on gfx950 FETCH_SIZE counts half the
bytes of a wide streaming read, so HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(MI355X_MICROARCH.md, HBM section).
"""
import json
import sys

# training-step stage name (vqhmm_elbo_stage_info) -> substring of the profiled kernel name
STEP = {
    "elbo_head": "elbo_head_pipe_kernel<3, 2, 8>",
    "strip_fwd(enc_conv1+enc_conv2+to_logits+dec_conv1+dec_conv2+to_params)": "strip_fwd_kernel<2, 0, 0>",
    "strip_fwd(enc_conv1+enc_conv2+to_logits+dec_conv1+dec_conv2+to_params+elbo_head)": "strip_fwd_kernel<2, 1, 0>",
    "strip_bwdw(to_params_dgrad+dec_conv2_dgrad+dec_conv1_dgrad+logits_bwd+to_logits_dgrad+enc_conv2_dgrad+6 wgrads)":
        "strip_bwdw_kernel<0>",
    "tail(slab reduction+composed dW/dE[+adam])": "tail_kernel<true>",
    "inputs_to_pcl+compose_fwd": "prologue_kernel",
}
# cfg4 dims (D = 16, K = 8: the round-3 launch chain, no strips): stage -> kernel
STEP_CFG4 = {
    "elbo_head": "elbo_head_coop_kernel<8, 2, 16, 8>",
    "enc_conv1+enc_conv2+to_logits": "conv2f_kernel<2, 1, 3, 1, false, 1>",
    "dec_conv1+dec_conv2+to_params": "conv2f_kernel<4, 2, 3, 1, false, 1>",
    "to_params_dgrad+dec_conv2_dgrad": "conv2f_kernel<4, 0, 1, 2, false, 2>",
    "dec_conv1_dgrad(+logits_bwd, to_logits_dgrad if K<=4)": "conv2w_kernel<1, 4, 3, 4, 0, false>",
    "enc_conv2_dgrad": "conv2w_kernel<4, 2, 3, 2, 0, false>",
    "wgrad_group(all 6 weight gradients)": "wgrad2_group_kernel<false>",
    "tail(slab reduction+composed dW/dE[+adam])": "tail_kernel<true>",
    "inputs_to_pcl+compose_fwd": "prologue_kernel",
}
# (bench.py section, kernel leg key) -> substring of the profiled kernel name
LEGS = {
    ("vq_cfg3", "vq_argmin"): "vq_rows_kernel<16, 2, false, 2, false>",
    ("viterbi_cfg5", "viterbi_cfg5"): "viterbi_kernel<8, true>",
    ("fwdbwd_cfg4", "fwdbwd_cfg4"): "fwdbwd_seg_kernel",
}


def _bytes(per_kernel, sub):
    hits = [v for k, v in per_kernel.items() if sub in k]
    if len(hits) != 1 or "FETCH_SIZE" not in hits[0] or "WRITE_SIZE" not in hits[0]:
        return None
    return round(2 * hits[0]["FETCH_SIZE"] * 1024 + hits[0]["WRITE_SIZE"] * 1024)


def main():
    srcs, dst = sys.argv[1:-1], sys.argv[-1]
    # sections not re-measured by this call keep their committed figures (merge into dst)
    try:
        out = {k: v for k, v in json.load(open(dst)).items() if not k.startswith("_")}
    except (OSError, ValueError):
        out = {}
    legs = {}
    for src in srcs:
        if "=" in src:  # a training-step pass at one (config, batch)
            sec, path = src.split("=", 1)
            per_kernel = json.load(open(path))
            out[sec] = {}
            for key, sub in (STEP_CFG4 if sec.startswith("cfg4") else STEP).items():
                v = _bytes(per_kernel, sub)
                if v is not None:
                    out[sec][key] = v
        else:
            legs.update(json.load(open(src)))
    for (sec, key), sub in LEGS.items():
        v = _bytes(legs, sub)
        if v is not None:
            out.setdefault(sec, {})[key] = v
    out["_note"] = ("HBM bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (rocprofv3 --pmc, separate passes, "
                    "gfx950 FETCH correction); this update's sources " + ", ".join(srcs))
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
