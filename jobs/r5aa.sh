set -o pipefail
mkdir -p gpurun_out/r5aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/r5aa/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --dtype fp32 --steps 100 --warmup 10 --stock_ref 1 > gpurun_out/r5aa/mlp32.log 2>&1
echo b rc=$?
timeout -k 10 300 python bench.py --dtype fp32 --steps 100 --warmup 10 --stock_ref 0 --no_fused_optimizer > gpurun_out/r5aa/mlp32_unfused.log 2>&1
echo b2 rc=$?
