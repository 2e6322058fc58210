# model parity tests + cfg2 step bench (no CPU baseline / HMM lines)
set -o pipefail
mkdir -p gpurun_out/step
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/step/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/step/pytest.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/step/pytest.log; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-hmm --steps 200 > gpurun_out/step/bench.json 2>gpurun_out/step/bench.err && \
python3 -c "
import json; d=json.load(open('gpurun_out/step/bench.json'))
print('ms_per_step', d['ms_per_step'], 'value', d['value']); print(json.dumps(d['step_kernels_us']))"
