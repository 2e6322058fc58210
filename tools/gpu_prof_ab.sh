# rocprofv3 kernel durations of the B=$B step under env variants: usage bash tools/gpu_prof_ab.sh TAG B "ENV1" "ENV2" ...
set -o pipefail
OUT=gpurun_out/$1; B=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for v in "$@"; do
  (cd /tmp && env $v timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $B --no-cpu-baseline --no-hmm --steps 20 --warmup 3 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/p$i.log 2>&1) || { tail -5 $OUT/p$i.log; exit 1; }
  echo "== $v"
  python3 tools/rocpd_stats.py $(find $OUT/p$i -name "*.db" | head -1) | grep -E "head|Name" | cut -c1-120
  i=$((i+1))
done
