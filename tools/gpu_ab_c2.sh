# A/B of two library builds on one box: the C2 bench alternately with each
# (tools/gpu_ab_c2.sh <variant .so> "<its RIO_EXTRA_FLAGS>" [rounds]); one JSON line per run in gpurun_out/ab_c2.jsonl
set -o pipefail
mkdir -p gpurun_out
B=${1:?variant library}
F=${2:?variant flags}
R=${3:-3}
: > gpurun_out/ab_c2.jsonl
for i in $(seq 1 $R); do
  for arm in new old; do
    if [ $arm = old ]; then export RIO_GPU_LIB=$B RIO_EXTRA_FLAGS="$F"; else unset RIO_GPU_LIB RIO_EXTRA_FLAGS; fi
    timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e > gpurun_out/ab_c2_run.json 2> gpurun_out/ab_c2_run.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_c2_run.json').read().strip().splitlines()[-1]); print(json.dumps({'arm':'$arm','round':$i,'ms_per_step':d['ms_per_step'],'value':d['value'],'one_context_ms':d.get('one_context',{}).get('ms_per_step'),'crc_ms':d['roofline']['kernel_ms']}))" >> gpurun_out/ab_c2.jsonl || exit 1
  done
done
unset RIO_GPU_LIB RIO_EXTRA_FLAGS
cat gpurun_out/ab_c2.jsonl
