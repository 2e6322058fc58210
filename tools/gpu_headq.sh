# head iteration: head / model / config GPU tests, the head's phase stamps, step times at B = 128 / 1024
set -o pipefail
OUT=gpurun_out/${1:-headq}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_model.py tests/test_gpu_configs.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
VQHMM_HEAD_PROF=1 timeout -k 10 200 python tools/conv_prof.py --head 128 1024 || exit 1
for b in 128 1024; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/b$b.json')); print($b, d['ms_per_step'], d['step_kernels_us'].get('elbo_head'))"
done
