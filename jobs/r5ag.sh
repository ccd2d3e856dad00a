set -o pipefail
mkdir -p gpurun_out/r5ag
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vgg.py -k "two_deep" tests/test_gpu_kernels.py::test_gemm_layouts > gpurun_out/r5ag/tests.log 2>&1
echo tests rc=$?
timeout -k 10 400 python benchmarks/conv_sweep.py --cfgs 6,8,13,14,15,21,22 --layers 1,2,3,4,5,6 --out gpurun_out/r5ag/sweep.json > gpurun_out/r5ag/sweep.log 2>&1
echo sweep rc=$?
