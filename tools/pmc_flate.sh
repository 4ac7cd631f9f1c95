#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short bench_flate run;
# counters per dispatch into gpurun_out/<name>_pN/. Args after the name go to
# bench_flate.py.
name=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d gpurun_out/${name}_p$i -o run -- \
    python3 -u tools/bench_flate.py --steps 1 --warmup 0 "$@" > gpurun_out/${name}_p$i.log 2>&1 || exit $?
  i=$((i+1))
done
