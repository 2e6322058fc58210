set -o pipefail
mkdir -p gpurun_out/h1
timeout -k 10 300 python -u -m pytest tests/test_gpu_hmm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/h1/pytest.log 2>&1; rc=$?
tail -25 gpurun_out/h1/pytest.log
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 120"
$T python tools/kbench.py viterbi --B 1024 --T 4096 --K 8 && $T python tools/kbench.py fwdbwd --B 512 --T 512 --K 8 && \
$T python tools/kbench.py viterbi --B 1024 --T 200 --K 3 && $T python tools/kbench.py fwdbwd --B 1024 --T 200 --K 3
