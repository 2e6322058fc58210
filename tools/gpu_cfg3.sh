# cfg3-dims iteration: the cfg3 / config GPU tests, the cfg3 bench (stage rooflines) and its rocprofv3 kernel
# stats.   usage: bash tools/gpu_cfg3.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-cfg3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 300 --timeout-method thread -k "cfg3 or configs" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py --config cfg3 --no-cpu-baseline --no-hmm --steps 10 --warmup 3 --profile-steps 3 > $OUT/cfg3.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --no-cpu-baseline --no-hmm --steps 5 --warmup 2 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof3.log 2>&1) || { tail -20 $OUT/prof3.log; exit 1; }
python3 tools/rocpd_stats.py $(find $OUT/prof3 -name "*.db" | head -1) --csv $OUT/cfg3_kernel_stats.csv > /dev/null
python3 - <<PY
import csv, json
d = json.load(open("$OUT/cfg3.json"))
print("cfg3", d["ms_per_step"], "ms", d["value"], "seq/s")
for k, v in d["stage_roofline"].items():
    print("   %-60s %9.1f us  %s %.3f" % (k[:60], v["us"], v["bound"], v["frac"]))
for r in list(csv.reader(open("$OUT/cfg3_kernel_stats.csv")))[1:16]:
    print("   %-70s %6s calls %10.1f us" % (r[0][:70], r[1], float(r[3]) / 1e3))
PY
