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
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_capture.py > gpurun_out/r5e/dist.log 2>&1
echo dist rc=$?
for v in 1 0; do
DDPX_SIDE_OPTIMIZER=$v timeout -k 10 300 python bench.py --gpus 1 --ddp_single --shard_optimizer 0 --bucket_plan default --steps 200 --warmup 20 > gpurun_out/r5e/ddp1_side$v.json 2>/dev/null || exit 1
done
echo ddp1 rc=$?
