# step A/B: serial backward vs side-stream weight gradients (bench.py, N=1, graph)
set -o pipefail
mkdir -p gpurun_out/ab
T="timeout -k 10 300"
$T python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "overlap or adam or train_model or cfg2" > gpurun_out/ab/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/ab/pytest.log
[ $rc -eq 0 ] || exit $rc
VQHMM_BWD_OVERLAP=0 $T python bench.py --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 > gpurun_out/ab/serial.json 2>gpurun_out/ab/serial.err && \
VQHMM_BWD_OVERLAP=1 $T python bench.py --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 > gpurun_out/ab/overlap.json 2>gpurun_out/ab/overlap.err && \
VQHMM_BWD_OVERLAP=0 $T python bench.py --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 --no-graph > gpurun_out/ab/serial_eager.json 2>>gpurun_out/ab/serial.err && \
VQHMM_BWD_OVERLAP=1 $T python bench.py --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 --no-graph > gpurun_out/ab/overlap_eager.json 2>>gpurun_out/ab/overlap.err && \
for f in serial overlap serial_eager overlap_eager; do python -c "import json,sys; d=json.load(open('gpurun_out/ab/$f.json')); print('$f', d['ms_per_step'], d['value'])"; done
