# strip-kernel check: its bit-identity tests + the golden / oracle model tests, then the step at
# B = 1024 and 128 with the strip launch on and off.   usage: bash tools/gpu_strip.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-strip}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_model.py tests/test_gpu_configs.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread -k "${2:-strip or golden or oracle or cfg}" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 128; do
  for v in 1 0; do
    VQHMM_STRIP=$v timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b${b}_s$v.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  done
done
python3 - <<PY
import json
for b in (1024, 128):
    for v in (1, 0):
        d = json.load(open("$OUT/b%d_s%d.json" % (b, v)))
        k = {n: t for n, t in d["step_kernels_us"].items() if not n.startswith("(")}
        print(b, "strip" if v else "pairs", d["ms_per_step"], json.dumps(k))
PY
