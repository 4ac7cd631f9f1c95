#!/bin/bash
# One GPU session of round 6: steps picked by the arguments, in order, each
# under its own time limit; stops at the first crash / abort / timeout (a plain
# test failure, rc 1, lets the later steps run). Output under gpurun_out/.
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
  tail -n 4 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name exited with $rc"
    exit $rc
  fi
  return 0
}

C2ONLY="--no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e"
while [ $# -gt 0 ]; do
  case "$1" in
    tests) step r06_pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread ;;
    smoke) step r06_smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step r06_bench 1100 python3 bench.py ;;
    c2) step r06_c2 300 python3 bench.py --steps 20 --warmup 5 $C2ONLY ;;
    profc2) step r06_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_c2 -o run -- \
        python3 bench.py --steps 10 --warmup 3 $C2ONLY ;;
    profc2_1) step r06_prof_c2_1ctx 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_c2_1ctx -o run -- \
        python3 bench.py --steps 10 --warmup 3 --c2-contexts 1 $C2ONLY ;;
    pmcc2)
      step r06_pmc_c2_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r06_pmc_c2_fetch -o run -- \
        python3 bench.py --steps 3 --warmup 1 $C2ONLY
      step r06_pmc_c2_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r06_pmc_c2_write -o run -- \
        python3 bench.py --steps 3 --warmup 1 $C2ONLY ;;
    prof1k) step r06_prof_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_c3 -o run -- \
        python3 tools/bench_flate.py --steps 2 ;;
    prof16k) step r06_prof_c3_16k 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_c3_16k -o run -- \
        python3 tools/bench_flate.py --per-block 16384 --steps 2 ;;
    profc4)
      [ -f /tmp/c4.bin ] || python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/r06_c4data.log 2>&1
      step r06_prof_c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof_c4 -o run -- \
        python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 2 ;;
    e2e) step r06_e2e 600 python3 tools/bench_e2e.py ;;
    c4p*)  # C4 alone, steps rotating over N context sets (c4p1: serial)
      [ -f /tmp/c4.bin ] || python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/r06_c4data.log 2>&1
      step r06_$1 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 4 --pipeline ${1#c4p} ;;
    ztests) step r06_ztests 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_zstd_gpu.py \
        tests/test_zstd_libzstd.py tests/test_chain_gpu.py tests/test_structural_fuzz_gpu.py -m gpu ;;
    pmcc4)  # FETCH_SIZE / WRITE_SIZE per kernel over a PMC_REPLICAS-replica C4 step (tools/pmc_summary.py)
      [ -f /tmp/c4.bin ] || python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/r06_c4data.log 2>&1
      for g in FETCH_SIZE WRITE_SIZE; do
        step r06_pmc_c4_$g 300 rocprofv3 --pmc $g --output-format csv -d gpurun_out/r06_pmc_c4_$g -o run -- \
          python3 -u tools/bench_zstd.py --data /tmp/c4.bin --steps 1 --warmup 0 --replicas ${PMC_REPLICAS:-8}
      done ;;
    pmcc3)
      for g in FETCH_SIZE WRITE_SIZE; do
        step r06_pmc_c3_$g 300 rocprofv3 --pmc $g --output-format csv -d gpurun_out/r06_pmc_c3_$g -o run -- \
          python3 -u tools/bench_flate.py --steps 1 --warmup 0 --replicas ${PMC_REPLICAS:-8}
      done ;;
    pmc16k)
      for g in FETCH_SIZE WRITE_SIZE; do
        step r06_pmc_c3_16k_$g 300 rocprofv3 --pmc $g --output-format csv -d gpurun_out/r06_pmc_c3_16k_$g -o run -- \
          python3 -u tools/bench_flate.py --steps 1 --warmup 0 --replicas ${PMC_REPLICAS:-8} --per-block 16384
      done ;;
    rehearse2)  # two ranks on the one GPU, collectives over gloo (bench.py REHEARSE sizes)
      step r06_rehearse2 900 env RIO_BENCH_REHEARSE=1 python3 bench.py --gpus 2 --steps 5 --warmup 2 ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
  shift
done
