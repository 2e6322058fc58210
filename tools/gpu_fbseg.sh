# Forward-backward iteration pass: the HMM GPU tests, then the cfg4-shard kernel time with the
# parallel-in-time kernel on / off, and its rocprofv3 kernel stats.   usage: bash tools/gpu_fbseg.sh TAG [K-EXPR]
set -o pipefail
OUT=gpurun_out/${1:-fbseg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hmm.py -x -q --tb=short --timeout 120 --timeout-method thread -k "${2:-forward_backward or gamma}" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for seg in 1 0; do
  for shape in "--B 512 --T 512 --K 8" "--B 4096 --T 512 --K 8" "--B 2048 --T 200 --K 8" "--B 512 --T 1024 --K 8"; do
    VQHMM_FB_SEG=$seg timeout -k 10 120 python tools/kbench.py fwdbwd $shape | sed "s/^/seg=$seg /" | tee -a $OUT/kbench.txt || exit 1
  done
done
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py fwdbwd --B 512 --T 512 --K 8 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1) || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/rocpd_stats.py $(find $OUT/prof -name "*.db" | head -1) --csv $OUT/kernel_stats.csv > /dev/null && cat $OUT/kernel_stats.csv | head -5
