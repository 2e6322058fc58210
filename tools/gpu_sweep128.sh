# B=128 step under the weight-gradient chunking and head grid knobs (A/B sweep, ms_per_step)
set -o pipefail
OUT=gpurun_out/sw128
mkdir -p $OUT
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --batch 128 --no-cpu-baseline --no-hmm --steps 300 --warmup 20 --profile-steps 0 > $OUT/$name.json 2>>$OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'])"
}
run base VQHMM_X=0
run small16 VQHMM_WGRAD_SMALL_CHUNKS=16
run small32 VQHMM_WGRAD_SMALL_CHUNKS=32
run small64 VQHMM_WGRAD_SMALL_CHUNKS=64
run minrows256 VQHMM_WGRAD_MINROWS=256
run minrows384 VQHMM_WGRAD_MINROWS=384
run min256_s32 VQHMM_WGRAD_MINROWS=256 VQHMM_WGRAD_SMALL_CHUNKS=32
run big96_s32 VQHMM_WGRAD_BIG_CHUNKS=96 VQHMM_WGRAD_SMALL_CHUNKS=32
run hgrid256 VQHMM_HEAD_GRID=256
run hgrid128 VQHMM_HEAD_GRID=128
run hgrid256_nbw2 VQHMM_HEAD_GRID=256 VQHMM_HEAD_NBW=2
run base2 VQHMM_X=0
