set -o pipefail
mkdir -p gpurun_out/r5aw
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5aw/gpu_suite.log 2>&1
echo suite rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5aw/vgg32.log 2>&1
echo b1 rc=$?
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5aw/deepnn32.log 2>&1
echo b2 rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5aw/vgg.log 2>&1
echo b3 rc=$?
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > gpurun_out/r5aw/deepnn.log 2>&1
echo b4 rc=$?
