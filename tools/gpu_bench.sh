# headline bench (N=1, strong/cfg2) + small-batch steps (the per-GPU batch of strong scaling at N=2,4,8)
# + a rocprofv3 kernel trace of the B=128 step.   usage: bash tools/gpu_bench.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-bench}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
for b in 512 256 128; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 200 > $OUT/bench_b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof128 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 128 --no-cpu-baseline --no-hmm --steps 50 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof128.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof128.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - <<PY
import json
for f in ["bench", "bench_b512", "bench_b256", "bench_b128"]:
    d = json.load(open("$OUT/%s.json" % f))
    print(f, d["config"]["per_gpu_batch"], "ms/step", d["ms_per_step"], "value", d["value"], "roof", (d.get("roofline") or {}).get("frac"))
d = json.load(open("$OUT/bench.json"))
print(json.dumps(d["cpu_baseline"]))
print(json.dumps(d["step_kernels_us"]))
PY
find $OUT/prof128 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -30'
