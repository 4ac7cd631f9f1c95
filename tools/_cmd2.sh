set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for c in same nocu copystream copystream_nocu; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/ce_$c -o run -- python3 tools/copy_engines2.py $c > gpurun_out/ce_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/ce_$c.log
  grep -c copyBuffer gpurun_out/ce_$c/*/run_kernel_trace.csv 2>/dev/null || grep -rc copyBuffer gpurun_out/ce_$c --include=run_kernel_trace.csv
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e > gpurun_out/c2_r05a.log 2>&1 || exit $?
tail -1 gpurun_out/c2_r05a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_two_contexts'], d['one_context'], d['parity']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_1ctx -o run -- python3 bench.py --steps 10 --warmup 3 --c2-contexts 1 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e > gpurun_out/prof_c2_1ctx.log 2>&1 || exit $?
tail -1 gpurun_out/prof_c2_1ctx.log | cut -c1-300
