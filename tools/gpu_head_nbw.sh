# head parity under both window sizes + head time at each batch for NBW = 1 / 4
set -o pipefail
mkdir -p gpurun_out/nbw
for n in 1 4; do
  VQHMM_HEAD_NBW=$n timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > gpurun_out/nbw/pytest_$n.log 2>&1 || { tail -30 gpurun_out/nbw/pytest_$n.log; exit 1; }
  echo "nbw=$n $(tail -1 gpurun_out/nbw/pytest_$n.log)"
done
for B in 128 256 512 1024; do for n in 1 4; do
  VQHMM_HEAD_NBW=$n timeout -k 10 60 python bench.py --batch $B --no-cpu-baseline --no-hmm --steps 100 --warmup 5 --profile-steps 8 > gpurun_out/nbw/b${B}_$n.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/nbw/b${B}_$n.json'));print($B, 'nbw', $n, 'head', d['step_kernels_us']['elbo_head'], 'step', d['ms_per_step'])"
done; done
