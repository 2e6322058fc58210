set -o pipefail
OUT=gpurun_out/pv1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_regimes.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python tools/infer_bench.py > $OUT/infer.log 2>&1 || { tail -20 $OUT/infer.log; exit 1; }
cat $OUT/infer.log
timeout -k 10 120 python tools/infer_bench.py 8192 512 >> $OUT/infer.log 2>&1 || { tail -20 $OUT/infer.log; exit 1; }
tail -1 $OUT/infer.log
