set -o pipefail
mkdir -p gpurun_out/r5bj
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f32.py -k "wino_wgrad or fp32" > gpurun_out/r5bj/tests.log 2>&1
echo tests rc=$?
DDPX_WINO_WGRAD_REDUCE=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f32.py -k "wino_wgrad" > gpurun_out/r5bj/tests2.log 2>&1
echo tests2 rc=$?
timeout -k 10 200 python benchmarks/wino_bench.py --only wgrad --out gpurun_out/r5bj/wgrad.json > gpurun_out/r5bj/wgrad.log 2>&1
echo bench rc=$?
DDPX_WINO_WGRAD_REDUCE=2 timeout -k 10 200 python benchmarks/wino_bench.py --only wgrad --out gpurun_out/r5bj/wgrad2.json > gpurun_out/r5bj/wgrad2.log 2>&1
echo bench2 rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bj/vgg32.log 2>&1
echo b1 rc=$?
