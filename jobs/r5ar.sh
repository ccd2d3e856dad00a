set -o pipefail
mkdir -p gpurun_out/r5ar
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/r5ar/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5ar/vgg32.log 2>&1
echo b1 rc=$?
DDPX_F32_WINO_WGRAD=0 timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ar/vgg32_direct_wgrad.log 2>&1
echo b2 rc=$?
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5ar/deepnn32.log 2>&1
echo b3 rc=$?
DDPX_F32_WINO_WGRAD=0 timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ar/deepnn32_direct_wgrad.log 2>&1
echo b4 rc=$?
