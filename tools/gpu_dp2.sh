# The N-rank bench path rehearsed with 2 ranks on this one GPU (gloo all-reduce; not a measurement).
set -o pipefail
OUT=gpurun_out/dp2
mkdir -p $OUT
VQHMM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-hmm --profile-steps 0 > $OUT/dp2.json 2> $OUT/dp2.err || { tail -20 $OUT/dp2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/dp2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['config']['parallelism'], d['ms_per_step'])"
