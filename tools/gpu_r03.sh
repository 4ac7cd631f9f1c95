#!/bin/bash
# One GPU session of round 3: steps picked by the arguments, in order, each
# under its own time limit; stops at the first crash / abort / timeout (a plain
# test failure, rc 1, lets the later steps run).
#   tests      smoke + pytest -m gpu
#   testsk K   pytest -m gpu -k K
#   c2         bench.py, C2 only
#   bench      bench.py, every config (no CPU baseline)
#   full       bench.py as the driver runs it
#   prof_c2    rocprofv3 kernel trace of the C2 bench
#   prof_all   rocprofv3 kernel trace of C2 + C3 + C5 (no CPU baseline)
#   pmc_c2     FETCH_SIZE / WRITE_SIZE passes over the C2 bench
#   ab_meta    C2 bench alternating the product library and exp_lib/nometa
#   enc_zstd / enc_flate   tools/bench_encode.py on the C3 records
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 12 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name exited with $rc"
    exit $rc
  fi
  return 0
}

C2="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-zstd --no-c5"
while [ $# -gt 0 ]; do
  case "$1" in
    tests)
      step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
      step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread ;;
    testsk)
      shift
      step pytest_k 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "$1" ;;
    c2) step c2 300 $C2 ;;
    bench) step bench 600 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    full) step full 900 python3 bench.py ;;
    prof_c2)
      step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-flate --no-zstd --no-c5 ;;
    prof_all)
      step prof_all 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_all -o run -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-zstd ;;
    pmc_c2)
      step pmc_c2_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c2_fetch -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-flate --no-zstd --no-c5
      step pmc_c2_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c2_write -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-flate --no-zstd --no-c5 ;;
    ab_meta)  # k_crc with the header checks (product) vs -DRIO_CRC_META=0 (exp_lib/nometa), alternating
      for i in 1 2; do
        step c2_meta_$i 300 $C2
        RIO_GPU_LIB=exp_lib/nometa/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_CRC_META=0" step c2_nometa_$i 300 $C2
      done ;;
    ab_ctx)  # C2 with steps alternating over 2 contexts (default) vs 1 context
      for i in 1 2; do
        step c2_ctx2_$i 300 $C2
        step c2_ctx1_$i 300 $C2 --c2-contexts 1
      done ;;
    enc_zstd) step enc_zstd 300 python3 tools/bench_encode.py --codec 2 ;;
    enc_flate) step enc_flate 300 python3 tools/bench_encode.py --codec 1 ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
  shift
done
