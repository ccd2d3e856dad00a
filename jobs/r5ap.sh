set -o pipefail
mkdir -p gpurun_out/r5ap
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vgg.py -k "two_deep" tests/test_gpu_kernels.py::test_gemm_layouts > gpurun_out/r5ap/tests.log 2>&1
echo tests rc=$?
timeout -k 10 400 python benchmarks/conv_sweep.py --cfgs 13,24 --layers 2,3,4,5,6 --out gpurun_out/r5ap/sweep.json > gpurun_out/r5ap/sweep.log 2>&1
echo sweep rc=$?
