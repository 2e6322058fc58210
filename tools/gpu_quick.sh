# model/step parity tests + bench at B=1024 and the strong-scaling per-GPU batches (no CPU baseline)
# usage: bash tools/gpu_quick.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_trainer.py -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 512 256 128; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/bench_b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
done
python3 - <<PY
import json
for b in (1024, 512, 256, 128):
    d = json.load(open("$OUT/bench_b%d.json" % b))
    print(b, "ms/step", d["ms_per_step"], "value", d["value"], "roof", d["roofline"]["kernel"], d["roofline"]["avg_us"], d["roofline"]["frac"])
    if b in (1024, 128):
        print("  ", json.dumps(d["step_kernels_us"]))
PY
