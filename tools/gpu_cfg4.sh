# cfg4 training step: one rank's shard (B=512) and the full 4096 at N=1, + rocprofv3 kernel stats of the shard
set -o pipefail
OUT=gpurun_out/${1:-cfg4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config cfg4 --batch 512 --no-cpu-baseline --no-hmm --steps 100 > $OUT/cfg4_b512.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-hmm --steps 50 > $OUT/cfg4_b4096.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof512 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --batch 512 --no-cpu-baseline --no-hmm --steps 30 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof512.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof512.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - <<PY
import json
for f in ["cfg4_b512", "cfg4_b4096"]:
    d = json.load(open("$OUT/%s.json" % f))
    print(f, d["config"]["per_gpu_batch"], "ms/step", d["ms_per_step"], "value", d["value"], "roof", json.dumps(d.get("roofline")))
    print(json.dumps(d["stage_roofline"]))
PY
find $OUT/prof512 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -30'
