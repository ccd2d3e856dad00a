set -o pipefail
mkdir -p gpurun_out/r5ae
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/r5ae/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/fp8_gemm_table.py --out gpurun_out/r5ae/fp8_table.json > gpurun_out/r5ae/fp8_table.txt 2>&1
echo table rc=$?
timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5ae/wide_fp8.log 2>&1
echo b1 rc=$?
DDPX_FP8_DGRAD=1 timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5ae/wide_fp8_dgrad.log 2>&1
echo b2 rc=$?
timeout -k 10 300 python bench.py --model mlp_wide --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5ae/wide_bf16.log 2>&1
echo b3 rc=$?
