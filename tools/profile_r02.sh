#!/bin/bash
# Round-2 profiles (the files committed under profiles/r02_*): per-config
# kernel traces (rocprofv3 --kernel-trace --stats) of the bench commands, then
# PMC passes, one rocprofv3 run per counter group (MI355X_MICROARCH.md slot
# limits), over shorter runs of the same benches. Output: gpurun_out/r02/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=${PROF_OUT:-gpurun_out/r02}
mkdir -p $O
timeout -k 10 200 python3 tools/bench_zstd.py --make-data --data /tmp/c4.rio > $O/c4data.log 2>&1 || exit $?
C2="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-flate --no-zstd --no-c5"
C3="python3 tools/bench_flate.py --steps 3"
C3K="python3 tools/bench_flate.py --steps 3 --per-block 16384"
C4="python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.rio"
kt() {  # kt <name> <cmd...>
  local name=$1; shift
  echo "=== kt $name ($(date +%T))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1
  local rc=$?; echo "=== kt $name rc=$rc"; return $rc
}
kt c2 $C2 && kt c3 $C3 && kt c3_16k $C3K && kt c4 $C4 || exit $?
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
SQB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
pm() {  # pm <name> <counters> <cmd...>
  local name=$1 ctr=$2; shift 2
  echo "=== pmc $name ($(date +%T))"
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$name -o run -- "$@" > $O/pmc_$name.log 2>&1
  local rc=$?; echo "=== pmc $name rc=$rc"; return $rc
}
C2P="python3 bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-flate --no-zstd --no-c5"
C3P="python3 tools/bench_flate.py --steps 1 --warmup 0 --replicas 8"
C4P="python3 tools/bench_zstd.py --steps 1 --warmup 0 --replicas 8 --data /tmp/c4.rio"
for cfg in c2 c3 c4; do
  case $cfg in c2) CMD=$C2P;; c3) CMD=$C3P;; c4) CMD=$C4P;; esac
  pm ${cfg}_fetch FETCH_SIZE $CMD && pm ${cfg}_write WRITE_SIZE $CMD && pm ${cfg}_sqa "$SQA" $CMD && pm ${cfg}_sqb "$SQB" $CMD || exit $?
  python3 tools/pmc_summary.py $O/pmc_${cfg}_fetch $O/pmc_${cfg}_write $O/pmc_${cfg}_sqa $O/pmc_${cfg}_sqb > $O/${cfg}_pmc.json
done
echo done
