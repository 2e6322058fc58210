# The step prologue's kernel time (rocprofv3 kernel trace, not event pairs) with its roles skipped by
# VQHMM_PRO_DBG bits (1 to_pcl x/u, 2 compose, 4 images, 8 head image, 16 count; results invalid, timing only),
# B = 128 and cfg2.  usage: bash tools/gpu_pro_dbg.sh
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prodbg
mkdir -p $OUT
for b in 128 1024; do for m in 0 1 6 31; do
  (cd /tmp && VQHMM_LIB_PATH=$GRAFT_REPO_ROOT/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so VQHMM_PRO_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/b${b}_m$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $b --no-cpu-baseline --no-hmm --steps 50 --warmup 5 --profile-steps 0 > $OUT/b${b}_m$m.log 2>&1) || { tail -5 $OUT/b${b}_m$m.log; exit 1; }
  db=$(find $OUT/b${b}_m$m -name "*.db" | head -1)
  python3 tools/rocpd_stats.py $db --csv $OUT/b${b}_m$m.csv > /dev/null && python3 - $OUT/b${b}_m$m.csv $b $m <<'PY'
import csv, sys
p = [r for r in csv.DictReader(open(sys.argv[1])) if "prologue" in r["Name"]]
print("B", sys.argv[2], "mask", sys.argv[3], "prologue avg us", round(float(p[0]["AverageNs"]) / 1e3, 2) if p else None)
PY
done; done
