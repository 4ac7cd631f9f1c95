#!/bin/bash
# Kernel-trace profile of a bench script: prof_bench.sh <name> <script.py> [args...]
# into gpurun_out/<name>/ (stats csv) and gpurun_out/<name>.bench.log.
name=$1; script=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- \
  python3 -u $script "$@" > gpurun_out/$name.bench.log 2>&1
