# step bench at one batch under a few env settings, on the profiling build (its knobs: csrc/common.h
# VQHMM_PROF_ENV), with rocprofv3 kernel averages: bash tools/gpu_ab_env_b.sh TAG BATCH "VAR=a" "VAR=b" ...
set -o pipefail
OUT=gpurun_out/$1; B=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  env VQHMM_LIB_PATH=$PWD/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so $e timeout -k 10 300 python bench.py --batch $B --no-cpu-baseline --no-hmm --steps 300 --profile-steps 0 > $OUT/b$i.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  (cd /tmp && env VQHMM_LIB_PATH=$GRAFT_REPO_ROOT/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch $B --no-cpu-baseline --no-hmm --steps 40 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof$i.log 2>&1) || { tail -20 $OUT/prof$i.log; exit 1; }
  python3 tools/rocpd_stats.py $(find $OUT/prof$i -name "*.db" | head -1) --csv $OUT/ks$i.csv > /dev/null
  python3 - <<PY
import csv, json
d = json.load(open("$OUT/b$i.json"))
ks = {r[0]: float(r[3]) / 1e3 for r in list(csv.reader(open("$OUT/ks$i.csv")))[1:]}
f = "${FILT:-wgrad,tail,strip,head,prologue}".split(",")
print("$e", "ms", d["ms_per_step"], {k.split("ILi")[0].split("ENS")[0][7:]: round(v, 1) for k, v in ks.items() if any(x in k for x in f)})
PY
done
