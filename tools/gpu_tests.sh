# full GPU test suite + smoke (one process each, bounded)
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=20 -v --tb=short --timeout 120 --timeout-method thread > gpurun_out/t/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t/pytest.log | tail -12
[ $rc -eq 0 ] || { tail -40 gpurun_out/t/pytest.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
