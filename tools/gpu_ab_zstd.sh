#!/bin/bash
# A/B of library variants on the C4 workload, alternating on one box:
#   tools/gpu_ab_zstd.sh <rounds> <name>=<flags> ...   ("base" = the product build)
# Variants are built beforehand with RIO_BUILD_DIR=exp_lib/<name> RIO_EXTRA_FLAGS=<flags>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
[ -f /tmp/c4.bin ] || python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/ab_c4data.log 2>&1 || exit 1
R=$1; shift
PIPE=${AB_PIPE:-2}
for r in $(seq 1 $R); do
  for v in "$@"; do
    name=${v%%=*}; fl=${v#*=}
    if [ "$name" = base ]; then
      timeout -k 10 300 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 4 --pipeline $PIPE > gpurun_out/ab_$name.log 2>&1 || exit $?
    else
      RIO_GPU_LIB=exp_lib/$name/librio_gpu.so RIO_EXTRA_FLAGS="$fl" timeout -k 10 300 \
        python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 4 --pipeline $PIPE > gpurun_out/ab_$name.log 2>&1 || exit $?
    fi
    tail -1 gpurun_out/ab_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'arm': '$name', 'round': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'serial': d['serial'] and d['serial']['value'], 'parity': d['parity']}))" | tee -a gpurun_out/ab_zstd.jsonl
  done
done
