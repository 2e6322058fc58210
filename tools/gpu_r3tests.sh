# selected GPU tests (one pytest process), bounded; args = pytest selection (default: every gpu test)
set -o pipefail
mkdir -p gpurun_out/t
[ $# -eq 0 ] && set -- tests -m gpu
timeout -k 10 900 python -u -m pytest "$@" -x -v --tb=short --timeout 300 --timeout-method thread > gpurun_out/t/pytest_sel.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t/pytest_sel.log | tail -30
[ $rc -eq 0 ] || tail -60 gpurun_out/t/pytest_sel.log
exit $rc
