set -o pipefail
OUT=gpurun_out/pvm
mkdir -p $OUT
for m in 0 1 2 3; do
VQHMM_PV_MODE=$m timeout -k 10 120 python tools/infer_bench.py > $OUT/infer_$m.log 2>&1; echo "mode $m"; tail -1 $OUT/infer_$m.log
done
