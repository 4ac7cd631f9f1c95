#!/bin/bash
# One GPU session of round 4: steps picked by the arguments, in order, each
# under its own time limit; stops at the first crash / abort / timeout (a plain
# test failure, rc 1, lets the later steps run).
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
  tail -n 6 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name exited with $rc"
    exit $rc
  fi
  return 0
}

c4data() {
  [ -f /tmp/c4.bin ] || python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1
}

PMC_SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
PMC_SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"

while [ $# -gt 0 ]; do
  case "$1" in
    smoke) step smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread ;;
    testsk) shift; step "pytest_$(echo "$1" | tr -c 'a-zA-Z0-9_' '_')" 600 \
        python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "$1" ;;
    testf) shift; step "pytest_$(basename "$1" .py)" 600 \
        python -u -m pytest "$1" -v --timeout 150 --timeout-method thread ;;
    c2) n_c2=$((n_c2 + 1)); step c2_$n_c2 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-flate16k --no-zstd \
        --no-c5 --no-e2e ;;
    c2v) shift; v=$1  # the C2 bench on an experiment build: exp_lib/<v>, its flags in exp_lib/<v>.flags
      n_c2v=$((n_c2v + 1))
      RIO_GPU_LIB=exp_lib/$v/librio_gpu.so RIO_EXTRA_FLAGS="$(cat exp_lib/$v.flags)" step c2_${v}_$n_c2v 300 \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e ;;
    c2v1) shift; v=$1; n_c2v=$((n_c2v + 1))  # the same, one context
      RIO_GPU_LIB=exp_lib/$v/librio_gpu.so RIO_EXTRA_FLAGS="$(cat exp_lib/$v.flags)" step c2c1_${v}_$n_c2v 300 \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e \
        --c2-contexts 1 ;;
    c2c1) step c2c1 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-flate --no-flate16k --no-zstd \
        --no-c5 --no-e2e --c2-contexts 1 ;;
    profc2) step profc2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc2 -o run -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e ;;
    b1k) step b1k 400 python3 tools/bench_flate.py --steps 3 ;;
    b1k_p2) step b1k_p2 400 python3 tools/bench_flate.py --steps 4 --pipeline 2 ;;
    b16k) step b16k 400 python3 tools/bench_flate.py --per-block 16384 --steps 3 ;;
    b16k_p2) step b16k_p2 400 python3 tools/bench_flate.py --per-block 16384 --steps 4 --pipeline 2 ;;
    c4) c4data; step c4 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 3 ;;
    c4_c2) c4data; step c4_c2 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 3 --contexts 2 ;;
    c4_p2) c4data; step c4_p2 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 4 --pipeline 2 ;;
    c5) step c5 600 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-e2e ;;
    bench) step bench 900 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchnc5) step benchnc5 900 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-e2e ;;
    e2e) c4data; step e2e 600 python3 tools/bench_e2e.py ;;
    full) step full 1100 python3 bench.py ;;
    prof16k) step prof16k 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16k -o run -- \
        python3 tools/bench_flate.py --per-block 16384 --steps 2 ;;
    prof1k) step prof1k 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1k -o run -- \
        python3 tools/bench_flate.py --steps 2 ;;
    profc4) c4data; step profc4 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc4 -o run -- \
        python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 2 ;;
    pmc16k)  # SQ counter passes over a 4-replica MaxItems-16384 run (one pass per group)
      step pmc16k_sq1 150 rocprofv3 --pmc $PMC_SQ1 --output-format csv -d gpurun_out/pmc16k_sq1 -o run -- \
        python3 -u tools/bench_flate.py --steps 1 --warmup 0 --replicas 8 --per-block 16384
      step pmc16k_sq2 150 rocprofv3 --pmc $PMC_SQ2 --output-format csv -d gpurun_out/pmc16k_sq2 -o run -- \
        python3 -u tools/bench_flate.py --steps 1 --warmup 0 --replicas 8 --per-block 16384 ;;
    pmc1k)
      step pmc1k_sq1 150 rocprofv3 --pmc $PMC_SQ1 --output-format csv -d gpurun_out/pmc1k_sq1 -o run -- \
        python3 -u tools/bench_flate.py --steps 1 --warmup 0 --replicas 8
      step pmc1k_sq2 150 rocprofv3 --pmc $PMC_SQ2 --output-format csv -d gpurun_out/pmc1k_sq2 -o run -- \
        python3 -u tools/bench_flate.py --steps 1 --warmup 0 --replicas 8 ;;
    pmcc2)  # FETCH_SIZE / WRITE_SIZE passes over the C2 bench (bench.py's roofline traffic)
      step pmc_c2_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c2_fetch -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e
      step pmc_c2_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c2_write -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-flate --no-flate16k --no-zstd --no-c5 --no-e2e ;;
    pmcc4)
      c4data
      step pmcc4_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcc4_fetch -o run -- \
        python3 -u tools/bench_zstd.py --data /tmp/c4.bin --steps 1 --warmup 0 --replicas 8
      step pmcc4_write 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcc4_write -o run -- \
        python3 -u tools/bench_zstd.py --data /tmp/c4.bin --steps 1 --warmup 0 --replicas 8 ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
  shift
done
