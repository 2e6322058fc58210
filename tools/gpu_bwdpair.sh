# backward pair (conv2g) on / off at cfg2, B=512, B=128
set -o pipefail
OUT=gpurun_out/bwp
mkdir -p $OUT
for b in 1024 512 128; do
  for rows in 1000000000 0; do
    VQHMM_BWD_PAIR_ROWS=$rows timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm > $OUT/b${b}_$rows.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b${b}_$rows.json')); k=d['step_kernels_us']; print('B=$b rows<$rows', d['ms_per_step'], {n: v for n, v in k.items() if ('dgrad' in n) and not n.startswith('(')})"
  done
done
