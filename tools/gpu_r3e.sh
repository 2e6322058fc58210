set -o pipefail
OUT=gpurun_out/r3e
mkdir -p $OUT
bash tools/gpu_r3tests.sh tests/test_gpu_head.py tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_trainer.py || exit 1
for b in 128 256 1024; do timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b$b.json || exit 1; done
for b in 128 1024; do VQHMM_HEAD=wave timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/b${b}_wave.json || exit 1; done
timeout -k 10 200 python bench.py --config cfg4 --batch 512 --no-cpu-baseline --no-hmm --steps 100 > $OUT/cfg4_b512.json || exit 1
python3 - <<PY
import json
for f in ["b128", "b128_wave", "b256", "b1024", "b1024_wave", "cfg4_b512"]:
    d = json.load(open("$OUT/%s.json" % f))
    print(f, d["ms_per_step"], "head", d["step_kernels_us"].get("elbo_head"), d["stage_roofline"].get("elbo_head"))
PY
