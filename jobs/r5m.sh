set -o pipefail
mkdir -p gpurun_out/r5m
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_dist.py > gpurun_out/r5m/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --ddp_single --stock_ref 0 > gpurun_out/r5m/ddp1.log 2>&1
echo bench rc=$?
