#!/bin/bash
# PMC passes on kernel micro-benchmarks (one counter group per rocprofv3 run).
set -o pipefail
OUT=gpurun_out/${1:-pmck}
mkdir -p $OUT
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
for what in "vq" "viterbi --B 1024 --T 4096 --K 8" "fwdbwd --B 512 --T 512 --K 8"; do
  tag=$(echo $what | cut -d' ' -f1)
  timeout -k 10 300 python tools/pmc.py --out $OUT/pmc_$tag.json --timeout 120 --groups "$SQ" "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/kbench.py $what > $OUT/pmc_$tag.log 2>&1 || { tail -20 $OUT/pmc_$tag.log; exit 1; }
  grep -v "^\[\|at::\|rocclr" $OUT/pmc_$tag.log | cut -c1-400
done
timeout -k 10 300 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/dist.log 2>&1; tail -4 $OUT/dist.log
timeout -k 10 200 python bench.py --no-graph --no-cpu-baseline --no-hmm --profile-steps 0 > $OUT/bench_eager.log 2>&1; tail -1 $OUT/bench_eager.log | cut -c1-300
