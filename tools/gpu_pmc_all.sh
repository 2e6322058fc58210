#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the cfg2 step (B = 1024 and the B = 128 shard) and the HMM/VQ kernel benches,
# then profiles-ready per-stage traffic.  usage: bash tools/gpu_pmc_all.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
for b in 1024 128; do
  timeout -k 10 400 python tools/pmc.py --out $OUT/pmc_step$b.json --timeout 150 --groups "$SQ" "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --batch $b --no-graph --steps 4 --warmup 1 --profile-steps 0 --no-hmm --no-cpu-baseline > $OUT/pmc_step$b.log 2>&1 || { tail -20 $OUT/pmc_step$b.log; exit 1; }
done
for what in "vq" "viterbi --B 1024 --T 4096 --K 8" "fwdbwd --B 512 --T 512 --K 8"; do
  tag=$(echo $what | cut -d' ' -f1)
  timeout -k 10 300 python tools/pmc.py --out $OUT/pmc_$tag.json --timeout 120 --groups "$SQ" "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/kbench.py $what > $OUT/pmc_$tag.log 2>&1 || { tail -20 $OUT/pmc_$tag.log; exit 1; }
done
python3 tools/make_pmc_traffic.py cfg2/B1024=$OUT/pmc_step1024.json cfg2/B128=$OUT/pmc_step128.json $OUT/pmc_vq.json $OUT/pmc_viterbi.json $OUT/pmc_fwdbwd.json $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
