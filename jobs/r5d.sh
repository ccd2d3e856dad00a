set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_kernels.py::test_linear_mlp_shapes_splitk" "tests/test_gpu_kernels.py::test_gemm_layouts" "tests/test_gpu_kernels.py::test_splitk_graph_replays" > gpurun_out/r5d/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/mlp_step_kernels.py --out gpurun_out/r5d/kernels.json > gpurun_out/r5d/kernels.txt 2>&1
echo bench rc=$?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py tests/test_gpu_multirank.py > gpurun_out/r5d/tests2.log 2>&1
echo tests2 rc=$?
