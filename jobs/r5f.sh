set -o pipefail
mkdir -p gpurun_out/r5f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_kernels.py::test_linear_mlp_shapes_splitk" "tests/test_gpu_kernels.py::test_gemm_layouts" > gpurun_out/r5f/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/mlp_step_kernels.py --out gpurun_out/r5f/kernels.json > gpurun_out/r5f/kernels.txt 2>&1
echo kernels rc=$?
timeout -k 10 300 python benchmarks/gemm_stamps.py --out gpurun_out/r5f/stamps.json > gpurun_out/r5f/stamps.txt 2>&1
echo stamps rc=$?
timeout -k 10 300 python benchmarks/window_probe.py --out gpurun_out/r5f/window.json > gpurun_out/r5f/window.txt 2>&1
echo window rc=$?
DDPX_SIDE_OPTIMIZER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/side1 -o run -- python bench.py --gpus 1 --ddp_single --shard_optimizer 0 --bucket_plan default --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5f/side1.log 2>&1
echo side1 rc=$?
DDPX_SIDE_OPTIMIZER=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/side0 -o run -- python bench.py --gpus 1 --ddp_single --shard_optimizer 0 --bucket_plan default --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5f/side0.log 2>&1
echo side0 rc=$?
timeout -k 10 300 python benchmarks/fp8_gemm_table.py --out gpurun_out/r5f/fp8_table.json > gpurun_out/r5f/fp8_table.txt 2>&1
echo fp8 rc=$?
