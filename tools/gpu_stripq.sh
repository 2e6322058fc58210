# quick strip-kernel iteration: its bit-identity tests, the phase profile, step times at B = 128 / 1024
set -o pipefail
OUT=gpurun_out/${1:-stripq}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread -k "${2:-strip}" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
VQHMM_STRIP_PROF=1 timeout -k 10 200 python tools/strip_prof.py 128 1024 || exit 1
VQHMM_STRIP_PROF=1 VQHMM_STRIP_BWD=0 timeout -k 10 200 python tools/strip_prof.py 128 || exit 1
for b in 128 1024; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/b$b.json')); k = {n: t for n, t in d['step_kernels_us'].items() if not n.startswith('(')}
print($b, d['ms_per_step'], json.dumps(k))"
done
