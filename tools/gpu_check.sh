#!/bin/bash
# One GPU session: smoke -> parity tests -> bench. Stops at the first crash,
# abort or timeout (a plain test failure, rc=1, still lets the bench run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export RIO_TEST_CODECS="${RIO_TEST_CODECS:-none,flate,zstd}"

step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name exited with $rc"
    exit $rc
  fi
  return 0
}

step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:---maxfail=8}
if [ -n "$ABLATE" ]; then
  step ablate 300 python tools/ablate.py
fi
if [ -n "$BENCH" ]; then
  step bench 300 python bench.py --steps 5 --warmup 2
fi
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
fi
if [ -n "$FLATE" ]; then
  step bench_flate 400 python tools/bench_flate.py ${FLATE_ARGS}
fi
