#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters (MI355X_MICROARCH.md
# "HBM / rocprofv3"): one rocprofv3 pass per counter group, then
# tools/pmc_summary.py averages per kernel (FETCH_SIZE doubled for the
# 16 B/lane streaming reads on gfx950, WRITE_SIZE as is) -> gpurun_out/pmc.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 bench.py --steps 3 --warmup 0 --no-cpu-baseline"}
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "=== pmc $ctr ($(date +%T))"
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_$ctr -o run -- $CMD \
    > gpurun_out/pmc_$ctr.log 2>&1
  rc=$?
  echo "=== pmc $ctr rc=$rc"
  tail -n 3 gpurun_out/pmc_$ctr.log
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc.json
cat gpurun_out/pmc.json
