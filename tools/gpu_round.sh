#!/bin/bash
# Round-end measurement session on one GPU: the default bench line, then
# rocprofv3 kernel-trace summaries of the same workloads (C2 + C3 through
# bench.py; C4 through tools/bench_zstd.py on a cached base file, since libzstd
# cannot be called under rocprofv3). Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
set -o pipefail
step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step bench 420 python bench.py
python tools/bench_zstd.py --make-data --data /tmp/c4.bin || exit 1
export TMPDIR=/tmp
step prof_c2c3 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2c3 -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-zstd
step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- \
  python3 tools/bench_zstd.py --replicas 80 --steps 3 --warmup 1 --data /tmp/c4.bin
