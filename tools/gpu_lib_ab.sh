# A/B of two builds of the library on the bench line: usage  bash tools/gpu_lib_ab.sh LIB_B BATCH...
# (alternating A = vqhmm/libvqhmm.so and B, twice each; prints ms/step and the dominant stage's time)
set -o pipefail
LB=$1; shift
mkdir -p gpurun_out/ab
for b in "$@"; do for rep in 1 2; do for lib in vq-vae-hmm-model_amd/vqhmm/libvqhmm.so $LB; do
  VQHMM_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > gpurun_out/ab/o.json 2>gpurun_out/ab/err || exit 1
  python - gpurun_out/ab/o.json $(basename $lib) $b <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print(sys.argv[3], sys.argv[2], d["ms_per_step"], {k[:12]: v for k, v in d["step_kernels_us"].items() if not k.startswith("(")})
PY
done; done; done
