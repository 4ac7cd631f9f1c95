set -o pipefail
mkdir -p gpurun_out
T=${1:-dyn}
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_encode_gpu.py -m gpu > gpurun_out/${T}_test.log 2>&1 && \
timeout -k 10 200 python tools/bench_encode.py --codec 1 --level 6 > gpurun_out/${T}_b6.json 2>&1 && \
timeout -k 10 200 python tools/bench_encode.py --codec 1 --level 1 > gpurun_out/${T}_b1.json 2>&1 && \
timeout -k 10 200 python tools/bench_encode.py --codec 2 > gpurun_out/${T}_bz.json 2>&1
