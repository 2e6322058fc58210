#!/bin/bash
# Kernel-level GPU pass: HMM kernels at cfg4/cfg5 per-GPU shapes, VQ launch-shape sweep, PMC HBM traffic.
set -o pipefail
OUT=gpurun_out/${1:-kern}
mkdir -p $OUT
export TMPDIR=/tmp
T="timeout -k 10 120"
$T python tools/kbench.py viterbi --B 1024 --T 4096 --K 8 > $OUT/hmm.jsonl && \
$T python tools/kbench.py fwdbwd --B 512 --T 512 --K 8 >> $OUT/hmm.jsonl && \
$T python tools/kbench.py viterbi --B 1024 --T 200 --K 3 >> $OUT/hmm.jsonl && \
$T python tools/kbench.py fwdbwd --B 1024 --T 200 --K 3 >> $OUT/hmm.jsonl && \
$T python tools/kbench.py stream >> $OUT/hmm.jsonl || exit 1
cat $OUT/hmm.jsonl
for pf in 1 0; do for w in 4 6 8 10 12 16; do
  echo -n "pf=$pf wpc=$w " >> $OUT/vq_sweep.txt
  VQHMM_VQ_PF=$pf VQHMM_VQ_WPC=$w $T python tools/kbench.py vq >> $OUT/vq_sweep.txt || exit 1
done; done
cat $OUT/vq_sweep.txt
timeout -k 10 400 python tools/pmc.py --out $OUT/pmc_step.json --timeout 150 --groups "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --no-cpu-baseline --no-graph --steps 3 --warmup 1 --profile-steps 0 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
cat $OUT/pmc.log | cut -c1-250
