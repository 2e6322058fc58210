# step time over batch sizes x env settings (graph, N=1, no profile/CPU/HMM lines)
# usage: bash tools/gpu_sweep.sh TAG "B1 B2 ..." "VAR=a" "VAR=b" ...   ("-" = no env)
set -o pipefail
OUT=gpurun_out/$1; BS=$2; shift 2
mkdir -p $OUT
for e in "$@"; do
  for b in $BS; do
    ev=""; [ "$e" != "-" ] && ev="$e"
    env $ev timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --profile-steps 0 --steps 300 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b.json'))
print('%-32s B=%-5d ms/step %.4f  seq/s %.0f' % ('$e', $b, d['ms_per_step'], d['value']))"
  done
done
