set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_scan_ahead_gpu.py tests/test_gpu_parity.py tests/test_structural_fuzz_gpu.py tests/test_gather_gpu.py tests/test_legacy.py -m gpu > gpurun_out/scan_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/scan_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 400 python3 tools/bench_e2e.py > gpurun_out/e2e_first$i.log 2>&1 || exit $?
tail -1 gpurun_out/e2e_first$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(' ', w['workload'], w['GiBs'], w['wall_ms'], w['spans'], w['parity']) for w in d['workloads']]"
done
