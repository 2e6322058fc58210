# SQ counters of the step's kernels at a given batch (default 128), one group per rocprofv3 pass
set -o pipefail
OUT=gpurun_out/${1:-pmc_head}
B=${2:-128}
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$OUT/counters.txt 2>&1) || true
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
timeout -k 10 300 python tools/pmc.py --out $OUT/pmc.json --timeout 120 --groups "$G1" "$G2" -- python3 bench.py --batch $B --no-graph --steps 3 --warmup 1 --profile-steps 0 --no-hmm --no-cpu-baseline > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
python3 - <<PY
import json
d = json.load(open("$OUT/pmc.json"))
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:12]:
    print(k[:70], {c: round(x) for c, x in v.items()})
PY
grep -i -E "mfma|SQ_INSTS" $OUT/counters.txt | head -40
