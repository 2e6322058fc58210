set -o pipefail
OUT=gpurun_out/ws3
mkdir -p $OUT
for b in 1024 128; do
for c in 128 256 512; do
  VQHMM_WGRAD_SMALL_CHUNKS=$c timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline --no-hmm --profile-steps 0 --steps 400 > $OUT/b${b}_s$c.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('B=$b small_chunks=$c', json.load(open('$OUT/b${b}_s$c.json'))['ms_per_step'])"
done
done
