# DP step form on one GPU (1-rank RCCL group): split graphs vs one graph with the collective inside,
# at B=128 and B=1024; then the 2-rank gloo rehearsal of the N-rank path (teardown exit codes)
set -o pipefail
OUT=gpurun_out/${1:-dpform}
mkdir -p $OUT
for b in 128 1024; do
  timeout -k 10 200 python bench.py --batch $b --dp-form --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 > $OUT/dp_split_b$b.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  VQHMM_DP_GRAPH=1 timeout -k 10 200 python bench.py --batch $b --dp-form --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 > $OUT/dp_graph_b$b.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --profile-steps 0 --steps 200 > $OUT/fused_b$b.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
python3 - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["ms_per_step"], d["config"]["step_form"], d["config"]["collective"])
PY
VQHMM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-hmm --profile-steps 0 > $OUT/dp2.json 2> $OUT/dp2.err; rc=$?
echo "dp2 rc=$rc"; grep -v amdgpu.ids $OUT/dp2.err | tail -5; cat $OUT/dp2.json
exit $rc
