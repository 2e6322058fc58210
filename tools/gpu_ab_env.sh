# step bench under a few env settings: bash tools/gpu_ab_env.sh TAG "VAR=a" "VAR=b" ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-hmm --steps 200 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json')); k=d['step_kernels_us']
print('$e', 'ms', d['ms_per_step'], {n: k[n] for n in k if 'wgrad' in n})"
done
