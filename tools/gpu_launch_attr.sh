# Launch-cost attribution at the B = 128 shard: the step's kernel trace with n empty
# launches inserted before the prologue / before the tail (profiling build, VQHMM_PRO_EMPTY /
# VQHMM_TAIL_EMPTY), and with the prologue's roles skipped (VQHMM_PRO_DBG=31); per-dispatch durations by
# predecessor (tools/launch_attr.py).   usage: bash tools/gpu_launch_attr.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-lattr}
mkdir -p $OUT
for v in "X=0" "VQHMM_PRO_EMPTY=1" "VQHMM_PRO_EMPTY=2" "VQHMM_TAIL_EMPTY=1" "VQHMM_PRO_EMPTY=1 VQHMM_PRO_DBG=31"; do
  tag=$(echo $v | tr ' =' '__')
  (cd /tmp && env $v VQHMM_LIB_PATH=$GRAFT_REPO_ROOT/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 128 --no-cpu-baseline --no-hmm --steps 40 --warmup 5 --profile-steps 0 > $OUT/$tag.log 2>&1) || { tail -5 $OUT/$tag.log; exit 1; }
  echo "== $v  $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log | tail -1)"
  python3 tools/launch_attr.py $(find $OUT/$tag -name "*.db" | head -1) | head -12
done
