set -o pipefail
mkdir -p gpurun_out/r5au
for v in s2w1o3 s2w1 s2w1o3; do
DDPX_WINO_WGRAD_VARIANT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f32.py -k "wino_wgrad" > gpurun_out/r5au/tests_$v.log 2>&1
echo tests $v rc=$?
DDPX_WINO_WGRAD_VARIANT=$v timeout -k 10 200 python benchmarks/wino_bench.py --only wgrad --out gpurun_out/r5au/wgrad_$v.json > gpurun_out/r5au/wgrad_$v.log 2>&1
echo bench $v rc=$?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f32.py -k "bn_relu_pool or fp32" > gpurun_out/r5au/tests_bn.log 2>&1
echo tests_bn rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5au/vgg32.log 2>&1
echo b1 rc=$?
DDPX_F32_BN_SPLIT=0 timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5au/vgg32_nosplit.log 2>&1
echo b2 rc=$?
