set -o pipefail
OUT=gpurun_out/wm
mkdir -p $OUT
for b in 1024 128; do
for w in 16 12 10 8; do
  VQHMM_CONV_WMAX=$w timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 400 > $OUT/b${b}_w$w.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b${b}_w$w.json')); k=d['step_kernels_us']; print('B=$b wmax=$w', d['ms_per_step'], {n[:24]: v for n, v in k.items() if 'conv' in n and not n.startswith('(')})"
done
done
