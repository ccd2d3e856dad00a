set -o pipefail
mkdir -p gpurun_out/r5e
timeout -k 10 300 python benchmarks/gemm_stamps.py --out gpurun_out/r5e/stamps.json > gpurun_out/r5e/stamps.txt 2>&1
echo stamps rc=$?
for i in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5e/ramp_$i.json 2>/dev/null || exit 1
DDPX_GRAPH_RAMP=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5e/noramp_$i.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/r5e/b200.json 2>/dev/null
echo bench rc=$?
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread "tests/test_gpu_multirank.py::test_native_sync_batchnorm_two_ranks_one_gpu" > gpurun_out/r5e/syncbn.log 2>&1
echo syncbn rc=$?
