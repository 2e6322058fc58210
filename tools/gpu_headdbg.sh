# head phase costs: elbo_head stage time with phases switched off (VQHMM_HEAD_DBG; results invalid)
set -o pipefail
OUT=gpurun_out/hd
mkdir -p $OUT
for b in ${BS:-1024 128}; do
  for m in ${MODES:-0 1 2 4 7 8}; do
    VQHMM_HEAD_DBG=$m timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 20 --warmup 3 > $OUT/b${b}_m$m.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b${b}_m$m.json')); print('B=$b dbg=$m head', d['step_kernels_us']['elbo_head'])"
  done
done
