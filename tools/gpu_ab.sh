# A/B of two library builds on one box: bench_encode alternately with each
set -o pipefail
mkdir -p gpurun_out
B=${1:-exp_lib/walk_scalar/librio_gpu.so}
shift
ARGS="$@"
for i in 1 2; do
  timeout -k 10 200 python tools/bench_encode.py $ARGS > gpurun_out/ab_new_$i.json 2>&1 || exit 1
  RIO_GPU_LIB=$B timeout -k 10 200 python tools/bench_encode.py $ARGS > gpurun_out/ab_old_$i.json 2>&1 || exit 1
done
