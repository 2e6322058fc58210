# the N-rank bench path rehearsed with 2 ranks on this one GPU (gloo all-reduce; not a measurement)
set -o pipefail
OUT=gpurun_out/dp2
mkdir -p $OUT
for i in 1 2 3; do
VQHMM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-hmm --profile-steps 0 > $OUT/dp2_$i.json 2> $OUT/dp2_$i.err; echo "rc=$?"
grep -v amdgpu.ids $OUT/dp2_$i.err | grep -v hostname | tail -5
done
python3 -c "import json; d=json.loads(open('$OUT/dp2_1.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['config']['parallelism'], d['ms_per_step'])"
