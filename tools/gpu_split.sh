#!/bin/bash
# Split copy pass session: its tests, the flate suites, C3 at MaxItems 16384
# with and without the split, C3 at 1024 per block. Stops at a crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log" | cut -c1-1200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited with $rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case "$s" in
    tests) step split_tests 600 python -u -m pytest tests/test_flate_split_gpu.py -x -v --timeout 150 --timeout-method thread ;;
    flate) step flate_tests 600 python -u -m pytest tests/test_flate_gpu.py tests/test_headline_gpu.py tests/test_chain_gpu.py -x -v --timeout 150 --timeout-method thread ;;
    all) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread ;;
    b16k) step b16k 400 python3 tools/bench_flate.py --per-block 16384 --steps 3 ;;
    b16k_ns) step b16k_ns 400 python3 tools/bench_flate.py --per-block 16384 --steps 3 --no-split ;;
    b1k) step b1k 400 python3 tools/bench_flate.py --steps 3 ;;
    prof16k) step prof16k 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16k -o run -- \
        python3 tools/bench_flate.py --per-block 16384 --steps 2 ;;
    stat1k) RIO_GPU_LIB=exp_lib/flstat/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_FLSTAT" RIO_BUILD_DIR=exp_lib/flstat \
        step stat1k 300 python3 tools/bench_flate.py --steps 1 --warmup 0 --replicas 4 ;;
    stat16k) RIO_GPU_LIB=exp_lib/flstat/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_FLSTAT" RIO_BUILD_DIR=exp_lib/flstat \
        step stat16k 300 python3 tools/bench_flate.py --steps 1 --warmup 1 --replicas 4 --per-block 16384 ;;
    nomerge) RIO_GPU_LIB=exp_lib/nomerge/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_SYNC_MERGE=1" RIO_BUILD_DIR=exp_lib/nomerge \
        step nomerge 300 python -u -m pytest tests/test_flate_gpu.py -x -v --timeout 150 --timeout-method thread ;;
    flate1) step flate1 300 python -u -m pytest tests/test_flate_gpu.py -x -v --timeout 150 --timeout-method thread ;;
    dbg) RIO_GPU_LIB=exp_lib/dbg/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_DEBUG_DUMP -DRIO_SYNC_DEBUG" RIO_BUILD_DIR=exp_lib/dbg \
        step dbg 300 python -u -m pytest "tests/test_flate_gpu.py::test_levels_and_styles" -x -s --timeout 150 --timeout-method thread ;;
    prof1k) step prof1k 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1k -o run -- \
        python3 tools/bench_flate.py --steps 2 ;;
    roots) for v in 10_8 11_8 12_8 10_9; do
          RIO_GPU_LIB=exp_lib/root$v/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_LIT_ROOT=${v%_*} -DRIO_DIST_ROOT=${v#*_}" \
            RIO_BUILD_DIR=exp_lib/root$v step b1k_root$v 300 python3 tools/bench_flate.py --steps 3
        done
        step b1k_base 300 python3 tools/bench_flate.py --steps 3 ;;
    ctx2) step b16k_c2 400 python3 tools/bench_flate.py --per-block 16384 --steps 3 --contexts 2
        step b1k_c2 400 python3 tools/bench_flate.py --steps 3 --contexts 2
        python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step c4_c1 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 3
        step c4_c2 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 3 --contexts 2 ;;
    ctxfix) step ctxchk 300 python3 tools/ctx_check.py --steps 3
        step ctxchk3 300 python3 tools/ctx_check.py --steps 2 --contexts 3
        step parse_tests 400 python -u -m pytest tests/test_contexts_gpu.py tests/test_parse_gpu.py tests/test_flate_gpu.py tests/test_headline_gpu.py -x -q --timeout 150 --timeout-method thread
        step b1k 400 python3 tools/bench_flate.py --steps 3
        step b1k_c2 400 python3 tools/bench_flate.py --steps 3 --contexts 2
        python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step c4_c2 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 3 --contexts 2
        step c4_c3 400 python3 tools/bench_zstd.py --data /tmp/c4.bin --steps 3 --contexts 3 ;;
    ctxchk) step ctxchk 300 python3 tools/ctx_check.py --steps 4
        step ctxchk_serial 300 python3 tools/ctx_check.py --steps 2 --serial ;;
    segw) for w in 10 14 24; do
          RIO_GPU_LIB=exp_lib/segw$w/librio_gpu.so RIO_BUILD_DIR=exp_lib/segw$w RIO_EXTRA_FLAGS="-DRIO_SEG_W10=$w" \
            step b16k_segw$w 400 python3 tools/bench_flate.py --per-block 16384 --steps 3
        done ;;
    ab_bitbuf) for i in 1 2; do
          step b1k_bitbuf_$i 300 python3 tools/bench_flate.py --steps 3
          RIO_GPU_LIB=exp_lib/nobitbuf/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_SYNC_BITBUF=0" RIO_BUILD_DIR=exp_lib/nobitbuf \
            step b1k_nobitbuf_$i 300 python3 tools/bench_flate.py --steps 3
        done ;;
    ab_exec2) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        for i in 1 2; do
          step c4_exec_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
          RIO_GPU_LIB=exp_lib/exec2/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZSTD_EXEC2=1" RIO_BUILD_DIR=exp_lib/exec2 \
            step c4_exec2_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        done ;;
    ab_zs2) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        for i in 1 2; do
          step c4_new_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
          RIO_GPU_LIB=exp_lib/zs2old/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZS2_PREFETCH=0 -DRIO_ZS2_CODES_ALU=0" \
            RIO_BUILD_DIR=exp_lib/zs2old step c4_old_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        done ;;
    ab_zs2b) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step c4_11 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        for v in 01 10 00; do
          RIO_GPU_LIB=exp_lib/zs2_$v/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZS2_PREFETCH=${v:0:1} -DRIO_ZS2_CODES_ALU=${v:1:1}" \
            RIO_BUILD_DIR=exp_lib/zs2_$v step c4_$v 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        done ;;
    profc4) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step profc4 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc4 -o run -- \
          python3 tools/bench_zstd.py --steps 2 --warmup 1 --data /tmp/c4.bin ;;
    zprof) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        RIO_GPU_LIB=exp_lib/zprof/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZPROF" RIO_BUILD_DIR=exp_lib/zprof \
          step zprof 300 python3 tools/bench_zstd.py --steps 1 --warmup 0 --replicas 8 --data /tmp/c4.bin ;;
    c4) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step c4 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin ;;
    norest) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step c4_base 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        RIO_GPU_LIB=exp_lib/norest/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZEXEC_NOREST=1" RIO_BUILD_DIR=exp_lib/norest \
          step c4_norest 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin ;;
    rmax) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        step c4_base 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        for v in 64 128 256; do
          RIO_GPU_LIB=exp_lib/rmax$v/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZEXEC_READY_MAX=$v" RIO_BUILD_DIR=exp_lib/rmax$v \
            step c4_rmax$v 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        done ;;
    ab_rp) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        for i in 1 2; do
          step c4_rp_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
          RIO_GPU_LIB=exp_lib/norp/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZEXEC_RESTPAR=0" RIO_BUILD_DIR=exp_lib/norp \
            step c4_norp_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        done ;;
    ab_pf) python3 tools/bench_zstd.py --make-data --data /tmp/c4.bin > gpurun_out/c4data.log 2>&1 || exit 1
        for i in 1 2; do
          step c4_pf2_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
          RIO_GPU_LIB=exp_lib/pf1/librio_gpu.so RIO_EXTRA_FLAGS="-DRIO_ZFIX_PF2=0" RIO_BUILD_DIR=exp_lib/pf1 \
            step c4_pf1_$i 300 python3 tools/bench_zstd.py --steps 3 --data /tmp/c4.bin
        done ;;
    zstdt) step zstd_tests 600 python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_libzstd.py -x -v --timeout 150 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
