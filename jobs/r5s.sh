set -o pipefail
mkdir -p gpurun_out/r5s
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "wino" tests/test_gpu_f32.py > gpurun_out/r5s/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/wino_bench.py --out gpurun_out/r5s/wino.json > gpurun_out/r5s/wino.txt 2>&1
echo wb rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5s/vgg32.log 2>&1
echo bench rc=$?
