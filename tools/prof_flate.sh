#!/bin/bash
# Kernel-trace profile of tools/bench_flate.py (args passed through) into
# gpurun_out/<name>/; prints the per-kernel stats.
name=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- \
  python3 -u tools/bench_flate.py --steps 3 "$@" > gpurun_out/$name.bench.log 2>&1 || exit $?
f=$(find gpurun_out/$name -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -12
