set -o pipefail
mkdir -p gpurun_out/wg
for n in 256 512 768 1024; do
  VQHMM_WGRAD_BIG_CHUNKS=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-hmm --steps 200 > gpurun_out/wg/b$n.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/wg/b$n.json')); k=d['step_kernels_us']
print($n, d['ms_per_step'], k['dec_conv2_wgrad'], k['enc_conv2_wgrad'], k['enc_conv1_wgrad'], k['dec_conv1_wgrad'], k['reduce_slabs'])"
done
