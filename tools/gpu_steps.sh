#!/bin/bash
# Run named GPU steps in order, each under its own time limit; stop at the first
# crash, abort or timeout (a plain failure, rc=1, lets later steps run).
#   bash tools/gpu_steps.sh "name:timeout:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; tmo=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log" | cut -c1-3000
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited with $rc"; exit $rc; fi
done
