"""Collect rocprofv3 PMC counters, one counter group per pass, and average them per kernel.

    python tools/pmc.py --out gpurun_out/pmc_vq.json --groups "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" \
        -- python3 tools/kbench.py vq

Each group is its own `rocprofv3 --pmc ... --kernel-trace` run (no sys/runtime tracing; the
program comes right after `--`).  This driver never touches the GPU itself.  Result: {kernel: {counter:
mean value per dispatch, "dispatches": n}}.  FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KB;
on gfx950 FETCH_SIZE reports half the bytes of a wide streaming read (MI355X_MICROARCH.md, HBM section),
so `hbm_bytes` = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 when both were collected.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict


def run_group(counters, cmd, workdir, tag, timeout):
    d = os.path.abspath(os.path.join(workdir, tag))
    os.makedirs(d, exist_ok=True)
    cmd = [os.path.abspath(c) if os.path.exists(c) else c for c in cmd]  # rocprofv3 runs from /tmp
    full = ["rocprofv3", "--pmc", *counters.split(), "--kernel-trace", "--output-format", "csv", "-d", d, "-o", tag,
            "--", *cmd]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(full, cwd="/tmp", env=env, timeout=timeout, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        raise SystemExit(f"rocprofv3 failed for group '{counters}' (rc={r.returncode})")
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(list))
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name") or row.get("Kernel-Name") or "?"
                acc[k][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
    out = {}
    for k, cs in acc.items():
        out[k] = {}
        for c, vals in cs.items():
            per = defaultdict(float)  # sum the per-instance rows of one dispatch
            for did, v in vals:
                per[did] += v
            out[k][c] = sum(per.values()) / len(per)
            out[k]["dispatches"] = len(per)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--groups", nargs="+", required=True)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    workdir = a.workdir or os.path.join(os.path.dirname(os.path.abspath(a.out)), "pmc_raw")
    merged = defaultdict(dict)
    for i, g in enumerate(a.groups):
        for k, cs in run_group(g, cmd, workdir, f"g{i}", a.timeout).items():
            merged[k].update(cs)
    for k, cs in merged.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            cs["hbm_bytes"] = 2 * cs["FETCH_SIZE"] * 1024 + cs["WRITE_SIZE"] * 1024
    with open(a.out, "w") as f:
        json.dump(merged, f, indent=1, sort_keys=True)
    for k, cs in merged.items():
        print(k[:90], json.dumps({c: round(v, 1) for c, v in cs.items()}))


if __name__ == "__main__":
    main()
