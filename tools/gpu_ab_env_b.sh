# step bench at one batch under a few env settings: bash tools/gpu_ab_env_b.sh TAG BATCH "VAR=a" "VAR=b" ...
set -o pipefail
OUT=gpurun_out/$1; B=$2; shift 2
mkdir -p $OUT
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --batch $B --no-cpu-baseline --no-hmm --steps 300 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json')); k=d['step_kernels_us']
print('$e', 'ms', d['ms_per_step'], {n[:12]: k[n] for n in k if any(f in n for f in '${FILT:-wgrad,tail}'.split(','))})"
done
