set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_gpu_dist.py::test_rccl_collectives" > gpurun_out/r5l/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/rccl_sweep.py --nproc 1 --protos default,Simple,LL --channels 0,4,16 --iters 5 --timeout 200 --out gpurun_out/r5l/sweep1.json > gpurun_out/r5l/sweep1.txt 2>&1
echo sweep rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --ddp_single --rccl_channels 8 --rccl_proto Simple --stock_ref 0 > gpurun_out/r5l/bench_ch8.log 2>&1
echo bench rc=$?
