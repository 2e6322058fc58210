# The round deliverable: full -m gpu suite + smoke, the bench line (cfg2 with CPU baseline and HMM kernel legs),
# the strong-scaling shard batches (B = 512 / 256 / 128 per GPU) and the DP step form at B = 128, rocprofv3
# kernel stats at cfg2 and B = 128.  PMC passes: tools/gpu_pmc_all.sh.   usage: bash tools/gpu_round.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-round}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
for b in 512 256 128; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/bench_b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
done
timeout -k 10 200 python bench.py --batch 128 --dp-form --no-cpu-baseline --no-hmm --steps 300 > $OUT/bench_b128_dpform.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
for b in 1024 128; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof$b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $b --no-cpu-baseline --no-hmm --steps 50 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof$b.log 2>&1) || { tail -20 $OUT/prof$b.log; exit 1; }
  python3 tools/rocpd_stats.py $(find $OUT/prof$b -name "*.db" | head -1) --csv $OUT/kernel_stats_b$b.csv > /dev/null
done
python3 - <<PY
import json
d = json.load(open("$OUT/bench.json"))
print(json.dumps({k: d[k] for k in ("value", "ms_per_step", "roofline", "cpu_baseline", "speedup_vs_cpu")})[:1500])
for f in ("bench_b512", "bench_b256", "bench_b128", "bench_b128_dpform"):
    e = json.loads([l for l in open("$OUT/%s.json" % f) if l.startswith("{")][-1])
    print(f, e["ms_per_step"], e["value"], e["config"]["step_form"])
PY
