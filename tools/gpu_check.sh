#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench line, rocprofv3 kernel stats of the bench.
# usage: bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json.log 2>&1 || { tail -20 $OUT/bench.json.log; exit 1; }
tail -1 $OUT/bench.json.log
R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/$OUT/bench_rocprof.log 2>&1 || { tail -20 $R/$OUT/bench_rocprof.log; exit 1; }
cd $R
find $OUT/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
echo done
