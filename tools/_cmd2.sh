set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
c2() {  # c2 <name> <lib> <flags>
  RIO_GPU_LIB=$2 RIO_EXTRA_FLAGS="$3" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e > gpurun_out/c2_$1.log 2>&1 || exit $?
  grep "^{" gpurun_out/c2_$1.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_two_contexts'], d['one_context']['ms_per_step'], d['parity']['ok'])"
}
for i in 1 2; do
  c2 base$i base_amd/lib/librio_gpu.so ""
  for v in w8b4 w10b4 w16b2 w12b2; do c2 ${v}_$i exp_lib/$v/librio_gpu.so "$(cat exp_lib/$v.flags)"; done
done
