# Iteration pass: a subset of the -m gpu suite (pytest -k EXPR, "" = all), then step times at cfg2 and B = 128
# with per-stage event times, and rocprofv3 kernel stats at both.   usage: bash tools/gpu_iter.sh TAG "EXPR"
set -o pipefail
OUT=gpurun_out/${1:-iter}
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1024 128; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/bench_b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof$b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $b --no-cpu-baseline --no-hmm --steps 50 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof$b.log 2>&1) || { tail -20 $OUT/prof$b.log; exit 1; }
  python3 tools/rocpd_stats.py $(find $OUT/prof$b -name "*.db" | head -1) --csv $OUT/kernel_stats_b$b.csv > /dev/null
  python3 - <<PY
import csv, json
e = json.load(open("$OUT/bench_b$b.json"))
print("B=$b", e["ms_per_step"], "ms", e["value"], "seq/s")
for r in list(csv.reader(open("$OUT/kernel_stats_b$b.csv")))[1:9]:
    print("   %-60s %8.1f us" % (r[0][:60], float(r[3]) / 1e3))
PY
done
