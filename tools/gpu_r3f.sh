set -o pipefail
OUT=gpurun_out/r3f
mkdir -p $OUT
bash tools/gpu_r3tests.sh tests/test_gpu_head.py tests/test_gpu_configs.py || exit 1
run() {  # name batch config env...
  local name=$1 b=$2 c=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --config $c --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/$name.json 2>>$OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], 'head', d['step_kernels_us'].get('elbo_head'))"
}
run cfg4 512 cfg4 VQHMM_X=0
run b128 128 cfg2 VQHMM_X=0
run b128_g256 128 cfg2 VQHMM_HEAD_GRID=256
run b128_g768 128 cfg2 VQHMM_HEAD_GRID=768
run b1024 1024 cfg2 VQHMM_X=0
run b1024_g768 1024 cfg2 VQHMM_HEAD_GRID=768
run b1024_g1024 1024 cfg2 VQHMM_HEAD_GRID=1024
run b1024_g256 1024 cfg2 VQHMM_HEAD_GRID=256
