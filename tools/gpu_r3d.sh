set -o pipefail
OUT=gpurun_out/r3d
mkdir -p $OUT
bash tools/gpu_r3tests.sh tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_head.py tests/test_gpu_trainer.py tests/test_gpu_regimes.py || exit 1
timeout -k 10 200 python bench.py --config cfg4 --batch 512 --no-cpu-baseline --no-hmm --steps 100 > $OUT/cfg4_b512.json || exit 1
for b in 128 1024; do timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b$b.json || exit 1; done
python3 - <<PY
import json
for f in ["cfg4_b512", "b128", "b1024"]:
    d = json.load(open("$OUT/%s.json" % f))
    print(f, d["ms_per_step"], {k: v for k, v in d["step_kernels_us"].items() if not k.startswith("(")})
PY
