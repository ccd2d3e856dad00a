set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 300 python benchmarks/capture_probe_torch.py > gpurun_out/r5c/capture_probe_torch.txt 2>&1
echo tprobe rc=$?
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_dist.py tests/test_gpu_entrypoints.py "tests/test_gpu_kernels.py::test_toy_mlp_fused_dgrad_step_bitwise" tests/test_gpu_vgg.py > gpurun_out/r5c/tests.log 2>&1
echo tests rc=$?
