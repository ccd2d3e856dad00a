set -o pipefail
mkdir -p gpurun_out/r5o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -k "wino" tests/test_gpu_f32.py > gpurun_out/r5o/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 10 --warmup 3 --stock_ref 0 > gpurun_out/r5o/vgg32_wino.log 2>&1
echo bench rc=$?
DDPX_F32_WINO=0 timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 10 --warmup 3 --stock_ref 0 > gpurun_out/r5o/vgg32_direct.log 2>&1
echo bench0 rc=$?
