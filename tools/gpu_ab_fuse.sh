# conv-pair fusion A/B: the step's GPU tests, then cfg2 / B=512 / B=128 steps with the fusion on / off
set -o pipefail
OUT=gpurun_out/fuse
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_model.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 512 128; do
  for t in 1 0; do
    VQHMM_CONV_FUSE=$t timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b${b}_f$t.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b${b}_f$t.json')); k=d['step_kernels_us']; print('B=$b fuse=$t', d['ms_per_step'], {n: v for n, v in k.items() if 'conv' in n and not n.startswith('(')})"
  done
done
