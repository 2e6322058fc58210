# tail_adam A/B: GPU tests for the step, then cfg2 and B=128 steps with the fused tail on / off
set -o pipefail
OUT=gpurun_out/tail
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_model.py tests/test_dist.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 128; do
  for t in 1 0; do
    VQHMM_TAIL_FUSED=$t timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b${b}_t$t.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b${b}_t$t.json')); print('B=$b tail_fused=$t', d['ms_per_step'])"
  done
done
# the N-rank bench path rehearsed with 2 ranks on this one GPU (gloo all-reduce; not a measurement)
VQHMM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-hmm > $OUT/dp2.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/dp2.json')); print('dp2 (gloo rehearsal)', d['n_gpus'], d['config']['per_gpu_batch'], d['ms_per_step'], d['config']['parallelism'])"
