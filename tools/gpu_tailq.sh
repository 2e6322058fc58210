# step tests + cfg2 / B=128 steps (tail changes)
set -o pipefail
OUT=gpurun_out/tq
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 128; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$b.json')); k=d['step_kernels_us']; print('B=$b', d['ms_per_step'], 'tail', k['tail(grad_tail+compose_bwd[+adam])'])"
done
