# ELBO head phase costs at B=128 and cfg2 (VQHMM_HEAD_DBG bits: 1 no A, 2 no B, 4 no C, 8 no windows,
# 32 no epilogue; results invalid, timings only) + the B=128 kernel stats
set -o pipefail
OUT=gpurun_out/${1:-hd128}
mkdir -p $OUT
export TMPDIR=/tmp
for b in 128 1024; do
for d in 0 8 1 2 4 5 32 40; do
  VQHMM_HEAD_DBG=$d timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 30 --warmup 5 --profile-steps 20 > $OUT/b${b}_d$d.json 2>>$OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b${b}_d$d.json')); print('B=$b dbg=$d', d['ms_per_step'], {k: v for k, v in d['step_kernels_us'].items() if not k.startswith('(')})"
done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof128 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 128 --no-cpu-baseline --no-hmm --steps 50 --profile-steps 0 > $GRAFT_REPO_ROOT/$OUT/prof128.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof128.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/rocpd_stats.py $(find $OUT/prof128 -name "*.db" | head -1) --csv $OUT/b128_kernel_stats.csv | cut -c1-150 | head -14
