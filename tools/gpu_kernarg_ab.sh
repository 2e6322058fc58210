# A/B of the HIP runtime's kernel-argument placement (HIP_FORCE_DEV_KERNARG=1: kernargs in device memory
# instead of host memory, so a dispatch's argument loads do not cross PCIe) on the step: B = 128 eager,
# B = 128 DP form, cfg2, alternating.   usage: bash tools/gpu_kernarg_ab.sh
set -o pipefail
for rep in 1 2; do
  for kv in 0 1; do
    for args in "--batch 128" "--batch 128 --dp-form" "--batch 1024"; do
      r=$(HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 120 python bench.py $args --no-cpu-baseline --no-hmm --steps 300 --profile-steps 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
      echo "DEV_KERNARG=$kv $args $r"
    done
  done
done
