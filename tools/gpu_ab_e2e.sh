#!/bin/bash
# A/B of scanner settings (environment variables) on the end-to-end bench,
# alternating on one box:  tools/gpu_ab_e2e.sh <rounds> <name>=<VAR=value,...> ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}
    env ${envs//,/ } timeout -k 10 400 python3 tools/bench_e2e.py ${AB_E2E_ARGS:-} > gpurun_out/abe_$name.log 2>&1 || exit $?
    tail -1 gpurun_out/abe_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'arm': '$name', 'env': '$envs', 'round': $r, 'rates': {w['workload']: w['GiBs'] for w in d['workloads']}, 'wall_ms': [w['wall_ms'] for w in d['workloads']], 'parity': d['parity']}))" | tee -a gpurun_out/ab_e2e.jsonl
  done
done
