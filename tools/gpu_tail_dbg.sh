# The fused tail's roles timed by skipping them (profiling build, VQHMM_TAIL_DBG bits: 1 segment reductions,
# 2 log_prior block, 4 loss finalize block, 8 Adam): B = 128 step and the tail stage.  Results invalid under a
# mask; timing only.  usage: bash tools/gpu_tail_dbg.sh
mkdir -p gpurun_out/taildbg
export VQHMM_LIB_PATH=$PWD/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so
for m in 0 1 2 4 6 8 15; do
  VQHMM_TAIL_DBG=$m timeout -k 10 200 python bench.py --batch 128 --no-cpu-baseline --no-hmm --steps 300 > gpurun_out/taildbg/m$m.json 2>gpurun_out/taildbg/err || exit 1
  python - gpurun_out/taildbg/m$m.json $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("mask", sys.argv[2], d["ms_per_step"], [v for k, v in d["step_kernels_us"].items() if k.startswith("tail")])
PY
done
