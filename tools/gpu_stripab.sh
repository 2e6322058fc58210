# A/B of the strip launches over the strong-scaling batch sizes: VQHMM_STRIP / VQHMM_STRIP_BWD on / off
set -o pipefail
OUT=gpurun_out/${1:-stripab}
mkdir -p $OUT
for b in 1024 512 256 128; do
  for v in "1 1" "1 0" "0 0"; do
    set -- $v
    VQHMM_STRIP=$1 VQHMM_STRIP_BWD=$2 timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/b${b}_$1$2.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    python3 -c "import json; d = json.load(open('$OUT/b${b}_$1$2.json')); print($b, 'fwd=$1 bwd=$2', d['ms_per_step'])"
  done
done
