# gradient accuracy vs the fp64 oracle (tools/grad_accuracy.py) at cfg4-shard and cfg2, default and
# with 4096 wgrad chunks (64-row slabs)
set -o pipefail
mkdir -p gpurun_out/gacc
T="timeout -k 10 300"
$T python tools/grad_accuracy.py > gpurun_out/gacc/cfg4.txt 2>&1 && \
VQHMM_WGRAD_CHUNKS=4096 $T python tools/grad_accuracy.py > gpurun_out/gacc/cfg4_4096.txt 2>&1 && \
$T python tools/grad_accuracy.py --dims 5,64,3,32,4,128 --B 1024 --T 200 > gpurun_out/gacc/cfg2.txt 2>&1 && \
VQHMM_WGRAD_CHUNKS=4096 $T python tools/grad_accuracy.py --dims 5,64,3,32,4,128 --B 1024 --T 200 > gpurun_out/gacc/cfg2_4096.txt 2>&1
rc=$?
for f in gpurun_out/gacc/*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
exit $rc
