# one iteration on the GPU box: full -m gpu suite (stops at the first failure), then step times at
# the strong-scaling per-GPU batches.   usage: bash tools/gpu_iter.sh TAG ["B1 B2 ..."]
set -o pipefail
OUT=gpurun_out/$1
BS=${2:-"1024 512 256 128"}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in $BS; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/bench_b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_b$b.json'))
print('B=%-5d ms/step %.4f seq/s %.0f  roof %s %.1fus %.3f' % ($b, d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['frac']))
print('   ', json.dumps({k: v for k, v in d['step_kernels_us'].items() if not k.startswith('(')}))"
done
