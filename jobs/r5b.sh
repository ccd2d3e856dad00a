set -o pipefail
mkdir -p gpurun_out/r5b
hipcc --offload-arch=gfx950 -O2 -std=c++17 benchmarks/capture_probe.hip -o gpurun_out/r5b/capture_probe -lpthread 2>/dev/null
timeout -k 10 60 gpurun_out/r5b/capture_probe > gpurun_out/r5b/capture_probe.txt 2>&1
echo probe rc=$?
timeout -k 10 300 python benchmarks/capture_probe_torch.py > gpurun_out/r5b/capture_probe_torch.txt 2>&1
echo tprobe rc=$?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_dist.py tests/test_gpu_entrypoints.py "tests/test_gpu_kernels.py::test_toy_mlp_fused_dgrad_step_bitwise" tests/test_gpu_vgg.py > gpurun_out/r5b/tests.log 2>&1
echo tests rc=$?
