#!/bin/bash
# Round-6 PMC passes: the cfg4 training step at its 8-GPU shard (B = 512) and full batch (B = 4096), the
# cfg2 step at B = 1024 and the B = 128 shard, and the forward-backward leg (now the segmented kernel),
# merged into profiles/pmc_traffic.json (other sections kept).   usage: bash tools/gpu_pmc_r6.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc6}
mkdir -p $OUT
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
run() {  # tag, bench args
  timeout -k 10 400 python tools/pmc.py --out $OUT/pmc_$1.json --timeout 150 --groups "$SQ" "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py $2 --no-graph --warmup 1 --profile-steps 0 --no-hmm --no-cpu-baseline > $OUT/pmc_$1.log 2>&1 || { tail -20 $OUT/pmc_$1.log; exit 1; }
}
run cfg4b512 "--config cfg4 --batch 512 --steps 4" && run cfg4b4096 "--config cfg4 --steps 2" && run cfg2b1024 "--batch 1024 --steps 4" && run cfg2b128 "--batch 128 --steps 4" || exit 1
timeout -k 10 300 python tools/pmc.py --out $OUT/pmc_fwdbwd.json --timeout 120 --groups "$SQ" "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/kbench.py fwdbwd --B 512 --T 512 --K 8 > $OUT/pmc_fwdbwd.log 2>&1 || { tail -20 $OUT/pmc_fwdbwd.log; exit 1; }
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
python3 tools/make_pmc_traffic.py cfg4/B512=$OUT/pmc_cfg4b512.json cfg4/B4096=$OUT/pmc_cfg4b4096.json cfg2/B1024=$OUT/pmc_cfg2b1024.json cfg2/B128=$OUT/pmc_cfg2b128.json $OUT/pmc_fwdbwd.json $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
