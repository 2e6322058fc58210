set -o pipefail
OUT=gpurun_out/ws2
mkdir -p $OUT
for c in 128 192 256 320 512; do
  VQHMM_WGRAD_BIG_CHUNKS=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-hmm --profile-steps 0 --steps 400 > $OUT/c$c.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('cfg2 big_chunks=$c', json.load(open('$OUT/c$c.json'))['ms_per_step'])"
done
for b in 512 256 128; do
for c in 256 512; do
for r in 128 192; do
  VQHMM_WGRAD_BIG_CHUNKS=$c VQHMM_WGRAD_MINROWS=$r timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline --no-hmm --profile-steps 0 --steps 400 > $OUT/b${b}_c${c}_r$r.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('B=$b big=$c minrows=$r', json.load(open('$OUT/b${b}_c${c}_r$r.json'))['ms_per_step'])"
done
done
done
