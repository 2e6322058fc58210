# per-stage times (bench.py step_kernels_us) of the N=1 step at batch B under a few env settings
# usage: bash tools/gpu_stage_ab.sh TAG B "VAR=a" "VAR=b" ...   ("-" = no env)
set -o pipefail
OUT=gpurun_out/$1; B=$2; shift 2
mkdir -p $OUT
for e in "$@"; do
  ev=""; [ "$e" != "-" ] && ev="$e"
  env $ev timeout -k 10 200 python bench.py --batch $B --no-cpu-baseline --no-hmm --steps 100 --profile-steps 10 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json'))
print('== $e  B=$B ms/step %.4f' % d['ms_per_step'])
print('   ', ', '.join('%s %.1f' % (k[:28], v) for k, v in d['step_kernels_us'].items() if not k.startswith('(')))"
done
