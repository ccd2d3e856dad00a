set -o pipefail
mkdir -p gpurun_out/r5am
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vgg.py -k "two_deep" tests/test_gpu_kernels.py::test_gemm_layouts > gpurun_out/r5am/tests.log 2>&1
echo tests rc=$?
timeout -k 10 400 python benchmarks/conv_sweep.py --cfgs 2,6,7,9,11,12,23 --layers 0,1 --out gpurun_out/r5am/sweep.json > gpurun_out/r5am/sweep.log 2>&1
echo sweep rc=$?
timeout -k 10 400 python benchmarks/conv_sweep.py --net deepnn --cfgs 6,7,23 --layers 1 --out gpurun_out/r5am/sweep_d.json > gpurun_out/r5am/sweep_d.log 2>&1
echo sweep2 rc=$?
