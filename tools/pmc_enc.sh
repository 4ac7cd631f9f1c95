#!/bin/bash
# SQ counters of the dynamic flate encoder (k_deflate_dyn): where its waves'
# cycles go (issue vs parked vs active), instruction mix, LDS conflicts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 tools/bench_encode.py --codec 1 --level 6 --reps 1 --replicas 8"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "=== pass $i ($(date +%T))"
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmce_$i -o run -- $CMD > gpurun_out/pmce_$i.log 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"
  tail -n 2 gpurun_out/pmce_$i.log
  [ $rc -eq 0 ] || exit $rc
done
