# Backward strip (with the folded weight gradients) above 2^17 rows: cfg2 step time with the profiling build's
# VQHMM_STRIP_BWD_ROWS raised, against the default, same box.   usage: bash tools/gpu_ab_rows.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-abrows}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=$PWD/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so
for b in 1024 512; do
  for rows in 131072 100000000 131072 100000000; do
    VQHMM_LIB_PATH=$LIB VQHMM_STRIP_BWD_ROWS=$rows timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 --profile-steps 0 > $OUT/b${b}_r$rows.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    python3 -c "import json; e=json.load(open('$OUT/b${b}_r$rows.json')); print('B=$b rows<$rows', e['ms_per_step'], 'ms')"
  done
done
