# PMC counters of every kernel of the step at batch B (default 1024 = cfg2), one group per
# rocprofv3 pass (SQ timing/instruction mix, then HBM bytes).   usage: bash tools/gpu_pmc_step.sh TAG [B]
set -o pipefail
OUT=gpurun_out/${1:-pmc_step}
B=${2:-1024}
mkdir -p $OUT
export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
G3="FETCH_SIZE"
G4="WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 400 python tools/pmc.py --out $OUT/pmc.json --timeout 90 --groups "$G1" "$G2" "$G3" "$G4" -- python3 bench.py --batch $B --no-graph --steps 3 --warmup 1 --profile-steps 0 --no-hmm --no-cpu-baseline > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
python3 - <<PY
import json
d = json.load(open("$OUT/pmc.json"))
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:24]:
    print(k[:90])
    print("   ", {c: round(x) for c, x in v.items()})
PY
