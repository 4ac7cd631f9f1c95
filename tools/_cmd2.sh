set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in 3 1 2; do
  if [ $v = 3 ]; then L=base_amd/lib/librio_gpu.so; F=""; else L=exp_lib/sdma$v/librio_gpu.so; F="$(cat exp_lib/sdma$v.flags)"; fi
  RIO_GPU_LIB=$L RIO_EXTRA_FLAGS="$F" timeout -k 10 400 python3 tools/bench_e2e.py > gpurun_out/e2e_sdmab$v.log 2>&1 || exit $?
  echo "RIO_SDMA=$v"; tail -1 gpurun_out/e2e_sdmab$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(' ', w['workload'], w['GiBs'], w['wall_ms'], w['parity']) for w in d['workloads']]"
done
