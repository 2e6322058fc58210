# The N-rank bench path rehearsed with 2 ranks on this one GPU (gloo all-reduce; not a measurement): bench.py's
# own spawn (--gpus 2) and the driver's torch.distributed.run launch; stdout must be exactly one JSON line.
set -o pipefail
OUT=gpurun_out/dp2
mkdir -p $OUT
check() { python3 -c "
import json, sys
lines = open(sys.argv[1]).read().strip().splitlines()
assert len(lines) == 1, 'stdout is not one line: %d lines' % len(lines)
d = json.loads(lines[0]); print(sys.argv[2], d['n_gpus'], d['config']['parallelism'], d['config']['step_form'], d['ms_per_step'])" $1 $2; }
VQHMM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-hmm --profile-steps 0 > $OUT/dp2.json 2> $OUT/dp2.err || { tail -20 $OUT/dp2.err; exit 1; }
check $OUT/dp2.json spawn || exit 1
VQHMM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-hmm --profile-steps 0 > $OUT/dp2_run.json 2> $OUT/dp2_run.err || { tail -20 $OUT/dp2_run.err; exit 1; }
check $OUT/dp2_run.json torchrun
