# HMM kernels on the GPU box: the -m gpu HMM tests, then bench.py's Viterbi / forward-backward
# lines under a few env settings.   usage: bash tools/gpu_fb.sh TAG "VAR=a" "VAR=b" ...  ("-" = no env)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hmm.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for e in "$@"; do
  ev=""; [ "$e" != "-" ] && ev="$e"
  env $ev timeout -k 10 200 python bench.py --batch 128 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json'))
for k in ('viterbi_cfg5', 'fwdbwd_cfg4'):
    r = d[k]; print('== $e %-13s %8.2f us  %7.1f GB/s  frac %.3f' % (k, r['avg_us'], r['achieved'], r['frac']))"
done
