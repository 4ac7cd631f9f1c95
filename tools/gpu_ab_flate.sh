#!/bin/bash
# A/B of library variants on the flate workloads, alternating on one box:
#   AB_PER_BLOCK=16384 AB_PIPE=1 tools/gpu_ab_flate.sh <rounds> <name>=<flags> ...   ("base" = the product build)
# Variants are built beforehand with RIO_BUILD_DIR=exp_lib/<name> RIO_EXTRA_FLAGS=<flags>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$1; shift
PB=${AB_PER_BLOCK:-1024}
PIPE=${AB_PIPE:-1}
for r in $(seq 1 $R); do
  for v in "$@"; do
    name=${v%%=*}; fl=${v#*=}
    if [ "$name" = base ]; then
      timeout -k 10 300 python3 tools/bench_flate.py --per-block $PB --steps 3 --pipeline $PIPE > gpurun_out/abf_$name.log 2>&1 || exit $?
    else
      RIO_GPU_LIB=exp_lib/$name/librio_gpu.so RIO_EXTRA_FLAGS="$fl" timeout -k 10 300 \
        python3 tools/bench_flate.py --per-block $PB --steps 3 --pipeline $PIPE > gpurun_out/abf_$name.log 2>&1 || exit $?
    fi
    tail -1 gpurun_out/abf_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'arm': '$name', 'per_block': $PB, 'round': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'serial': d['serial'] and d['serial']['value'], 'parity': d['parity'], 'stage_ms': d['stage_ms']}))" | tee -a gpurun_out/ab_flate.jsonl
  done
done
