#!/bin/bash
# Round-3 profile session: kernel-trace summaries of the bench configs (C2 + C3
# + C5 through bench.py, C4 through tools/bench_zstd.py on a cached base file,
# C3 at MaxItems 16384) and the flate PMC passes. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
step prof_c2c3c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2c3c5 -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-zstd
step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- \
  python3 tools/bench_zstd.py --steps 3 --warmup 1 --data /tmp/c4.bin
step prof_c3_16k 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_16k -o run -- \
  python3 tools/bench_flate.py --per-block 16384 --steps 3
step pmc_c3 600 bash tools/pmc_flate.sh pmc_c3 --replicas 8
