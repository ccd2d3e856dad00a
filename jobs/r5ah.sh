set -o pipefail
mkdir -p gpurun_out/r5ah
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vgg.py tests/test_gpu_kernels.py::test_gemm_layouts > gpurun_out/r5ah/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ah/vgg_new.log 2>&1
echo b1 rc=$?
DDPX_CONV_PICKS=r4 timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ah/vgg_r4.log 2>&1
echo b2 rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ah/vgg_new2.log 2>&1
echo b3 rc=$?
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > gpurun_out/r5ah/deepnn_new.log 2>&1
echo b4 rc=$?
DDPX_CONV_PICKS=r4 timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > gpurun_out/r5ah/deepnn_r4.log 2>&1
echo b5 rc=$?
timeout -k 10 400 python benchmarks/conv_sweep.py --cfgs 5,14,15,21,22 --layers 6 --out gpurun_out/r5ah/sweep_4x4.json > gpurun_out/r5ah/sweep_4x4.log 2>&1
echo s1 rc=$?
timeout -k 10 400 python benchmarks/conv_sweep.py --net deepnn --cfgs 5,6,7,8,12,13,15,21,22 --out gpurun_out/r5ah/sweep_deepnn.json > gpurun_out/r5ah/sweep_deepnn.log 2>&1
echo s2 rc=$?
