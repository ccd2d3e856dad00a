set -o pipefail
mkdir -p gpurun_out/r5n
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_kernels.py::test_linear_mlp_shapes_splitk" "tests/test_gpu_kernels.py::test_gemm_layouts" > gpurun_out/r5n/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/gemm_stamps.py --out gpurun_out/r5n/stamps.json > gpurun_out/r5n/stamps.txt 2>&1
echo stamps rc=$?
timeout -k 10 300 python benchmarks/mlp_step_kernels.py --out gpurun_out/r5n/kernels.json > gpurun_out/r5n/kernels.txt 2>&1
echo kernels rc=$?
