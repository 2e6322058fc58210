# rocprofv3 kernel-trace stats of the graphed step at batch B under a few env settings
# usage: bash tools/gpu_trace_ab.sh TAG B "VAR=a" "VAR=b" ...   ("-" = no env)
set -o pipefail
OUT=gpurun_out/$1; B=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for e in "$@"; do
  ev=""; [ "$e" != "-" ] && ev="$e"
  d=$GRAFT_REPO_ROOT/$OUT/t$i
  (cd /tmp && env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $B --no-cpu-baseline --no-hmm --steps 50 --profile-steps 0 > $d.log 2>&1) || { tail -20 $d.log; exit 1; }
  echo "== $e"
  python3 tools/rocpd_stats.py $(find $d -name "*.db" | head -1) | cut -c1-150 | head -24
  i=$((i+1))
done
