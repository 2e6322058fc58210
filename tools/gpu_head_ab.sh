# head-stage time under experiment skip bits (VQHMM_HEAD_DBG), B=128 and B=1024
set -o pipefail
mkdir -p gpurun_out/hab
for B in 128 1024; do for d in 0 1 2 4 8 16 6 7 15 31; do
  VQHMM_HEAD_DBG=$d timeout -k 10 60 python bench.py --batch $B --no-cpu-baseline --no-hmm --steps 5 --warmup 2 --profile-steps 8 > gpurun_out/hab/b${B}_$d.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hab/b${B}_$d.json'));print($B, $d, d['step_kernels_us']['elbo_head'])"
done; done
