set -o pipefail
OUT=gpurun_out/hs
mkdir -p $OUT
for b in 1024 512 256 128; do
for n in 1 2 4; do
  VQHMM_HEAD_NBW=$n timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline --no-hmm --profile-steps 0 --steps 400 > $OUT/b${b}_n$n.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('B=$b nbw=$n', json.load(open('$OUT/b${b}_n$n.json'))['ms_per_step'])"
done
done
