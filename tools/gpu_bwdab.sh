# backward strip: its identity tests, then the step with the strip on (any size) / off at B = 1024, 512, 128
set -o pipefail
OUT=gpurun_out/${1:-bwdab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread -k strip_backward > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 512 128; do
  for v in "1 999999999" "0 0"; do
    set -- $v
    VQHMM_STRIP_BWD=$1 VQHMM_STRIP_BWD_ROWS=$2 timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/b${b}_$1.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    python3 -c "import json; d = json.load(open('$OUT/b${b}_$1.json')); print($b, 'strip_bwd=$1', d['ms_per_step'])"
  done
done
