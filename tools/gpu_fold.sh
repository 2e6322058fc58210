# Fold iteration pass: the fold / strip / DP tests, phase stamps of the folded backward strip (profiling build)
# at B = 128 / 256 / 512, and step times at B = 128 / 256 / 512 / 1024.   usage: bash tools/gpu_fold.sh TAG ["EXPR"]
set -o pipefail
OUT=gpurun_out/${1:-fold}
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:-fold or strip_backward or shards or fused_tail}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
VQHMM_LIB_PATH=$PWD/vq-vae-hmm-model_amd/vqhmm/libvqhmm_prof.so VQHMM_STRIP_PROF=1 timeout -k 10 200 python tools/bwdw_prof.py 128 256 512 2>&1 | grep -v amdgpu.ids | tee $OUT/bwdw_prof.txt
for b in 128 256 512 1024; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 300 > $OUT/bench_b$b.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json; e=json.load(open('$OUT/bench_b$b.json')); print('B=$b', e['ms_per_step'], 'ms', e['value'], 'seq/s')"
done
