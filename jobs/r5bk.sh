set -o pipefail
mkdir -p gpurun_out/r5bk
DDPX_WINO_TK=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f32.py -k "wino or fp32 or deepnn" > gpurun_out/r5bk/tests16.log 2>&1
echo tests16 rc=$?
timeout -k 10 300 python benchmarks/wino_bench.py --out gpurun_out/r5bk/l32.json > gpurun_out/r5bk/l32.log 2>&1
echo b32 rc=$?
DDPX_WINO_TK=16 timeout -k 10 300 python benchmarks/wino_bench.py --out gpurun_out/r5bk/l16.json > gpurun_out/r5bk/l16.log 2>&1
echo b16 rc=$?
DDPX_WINO_TK=16 timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bk/v16.log 2>&1
echo v16 rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bk/v32.log 2>&1
echo v32 rc=$?
