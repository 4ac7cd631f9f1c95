set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_encode_gpu.py -m gpu > gpurun_out/dyn_test.log 2>&1 && \
timeout -k 10 200 python tools/bench_encode.py --codec 1 --level 1 > gpurun_out/dyn_b1.json 2>&1 && \
timeout -k 10 200 python tools/bench_encode.py --codec 1 --level 6 > gpurun_out/dyn_b6.json 2>&1
