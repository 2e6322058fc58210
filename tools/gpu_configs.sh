# training step at the other BASELINE configs, N=1: cfg4 (full 4096 and one rank's 512), cfg3 dims (B=2048),
# with rocprofv3 kernel stats of cfg4 (the B=512 shard: cfg4_kernel_stats.csv; B=4096: cfg4f_) and of cfg3
set -o pipefail
OUT=gpurun_out/${1:-cfgs}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-hmm --steps 30 --warmup 5 > $OUT/cfg4_b4096.json 2>>$OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
timeout -k 10 300 python bench.py --config cfg4 --batch 512 --no-cpu-baseline --no-hmm --steps 100 > $OUT/cfg4_b512.json 2>>$OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
timeout -k 10 300 python bench.py --config cfg4 --batch 512 --dp-form --no-cpu-baseline --no-hmm --steps 100 > $OUT/cfg4_b512_dpform.json 2>>$OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
timeout -k 10 400 python bench.py --config cfg3 --no-cpu-baseline --no-hmm --steps 10 --warmup 3 --profile-steps 3 > $OUT/cfg3_b2048.json 2>>$OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 - <<PY
import json
for f in ["cfg4_b4096", "cfg4_b512", "cfg4_b512_dpform", "cfg3_b2048"]:
    d = json.load(open("$OUT/%s.json" % f))
    print(f, d["ms_per_step"], d["value"], json.dumps(d["roofline"]))
    print("  ", {k: v for k, v in d["step_kernels_us"].items() if not k.startswith("(")})
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --batch 512 --no-cpu-baseline --no-hmm --steps 30 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof4.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof4f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --no-cpu-baseline --no-hmm --steps 10 --warmup 3 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof4f.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof4f.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --no-cpu-baseline --no-hmm --steps 5 --warmup 2 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof3.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof3.log; exit 1; }
cd $GRAFT_REPO_ROOT
for c in 4 4f 3; do python3 tools/rocpd_stats.py $(find $OUT/prof$c -name "*.db" | head -1) --csv $OUT/cfg${c}_kernel_stats.csv > $OUT/cfg${c}_stats.txt; cut -c1-140 $OUT/cfg${c}_stats.txt | head -12; done
