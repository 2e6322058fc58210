# wgrad chunking sweep on the current step (cfg2: big-output chunks; B=128: minimum rows per chunk)
set -o pipefail
OUT=gpurun_out/ws
mkdir -p $OUT
for c in 256 384 512 768 1024; do
  VQHMM_WGRAD_BIG_CHUNKS=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-hmm --profile-steps 0 --steps 400 > $OUT/c$c.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('cfg2 big_chunks=$c', json.load(open('$OUT/c$c.json'))['ms_per_step'])"
done
for r in 64 128 192 256; do
  VQHMM_WGRAD_MINROWS=$r timeout -k 10 120 python bench.py --batch 128 --no-cpu-baseline --no-hmm --profile-steps 0 --steps 400 > $OUT/r$r.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('B=128 minrows=$r', json.load(open('$OUT/r$r.json'))['ms_per_step'])"
done
