#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (one rocprofv3 run each) over a short C4 run:
# counters per dispatch into gpurun_out/<name>_pN/.
name=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/${name}_data.log 2>&1 || exit 1
i=0
for g in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d gpurun_out/${name}_p$i -o run -- \
    python3 -u tools/bench_zstd.py --steps 1 --warmup 0 --replicas 8 --data /tmp/c4.bin "$@" > gpurun_out/${name}_p$i.log 2>&1 || exit $?
  i=$((i+1))
done
