# rocprofv3 kernel stats of one bench configuration: bash tools/gpu_prof1.sh TAG BENCH-ARGS...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-hmm --steps 50 --profile-steps 0 "$@" > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1) || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/rocpd_stats.py $(find $OUT/prof -name "*.db" | head -1) --csv $OUT/kernel_stats.csv > /dev/null
grep -v '^{' $OUT/prof.log | grep -iv "amdgpu.ids\|hostname\|gloo" | tail -3
python3 - <<PY
import csv, json
for l in open("$OUT/prof.log"):
    if l.startswith("{"):
        e = json.loads(l); print("$*", e["ms_per_step"], "ms", e["value"], "seq/s", e["config"]["step_form"])
for r in list(csv.reader(open("$OUT/kernel_stats.csv")))[1:12]:
    print("   %-70s %6s calls %8.1f us" % (r[0][:70], r[1], float(r[3]) / 1e3))
PY
