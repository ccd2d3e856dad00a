set -o pipefail
mkdir -p gpurun_out/r5x
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x/gpu_suite.log 2>&1
echo suite rc=$?
