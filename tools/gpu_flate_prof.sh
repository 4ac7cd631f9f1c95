set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_encode_gpu.py -m gpu > gpurun_out/fp_test.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -o run -- python tools/bench_encode.py --codec 1 --level 6 --reps 3 > gpurun_out/fp_b6.json 2> gpurun_out/fp_prof.err
