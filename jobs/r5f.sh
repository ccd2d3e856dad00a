set -o pipefail
mkdir -p gpurun_out/r5f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/window_probe.py --out gpurun_out/r5f/window.json > gpurun_out/r5f/window.txt 2>&1
echo window rc=$?
DDPX_SIDE_OPTIMIZER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/side1 -o run -- python bench.py --gpus 1 --ddp_single --shard_optimizer 0 --bucket_plan default --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5f/side1.log 2>&1
echo side1 rc=$?
DDPX_SIDE_OPTIMIZER=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/side0 -o run -- python bench.py --gpus 1 --ddp_single --shard_optimizer 0 --bucket_plan default --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5f/side0.log 2>&1
echo side0 rc=$?
