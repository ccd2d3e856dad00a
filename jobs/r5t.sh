set -o pipefail
mkdir -p gpurun_out/r5t
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/r5t/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5t/dnn32.log 2>&1
echo bench rc=$?
DDPX_F32_WINO=0 timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5t/dnn32_direct.log 2>&1
echo bench0 rc=$?
