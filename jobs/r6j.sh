set -o pipefail
mkdir -p gpurun_out/r6j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6j
export MASTER_ADDR=127.0.0.1
timeout -k 10 200 python benchmarks/deepnn_tile_probe.py > $O/tiles.log 2>&1 && echo tiles ok &&
for N in 2 4 8; do for Z in 0 1; do
  timeout -k 10 200 python bench.py --gpus 1 --ddp_single --sim_world $N --shard_optimizer $Z --bucket_plan default --steps 200 --warmup 20 --stock_ref 0 > $O/sim${N}_z${Z}.log 2>&1 || exit 1
done; done && echo sim ok &&
timeout -k 10 200 python bench.py --gpus 1 --ddp_single --steps 200 --warmup 20 --stock_ref 0 --bucket_plan default --shard_optimizer 0 > $O/sim1_z0.log 2>&1 && echo sim1 ok &&
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --stock_ref 0 > $O/single.log 2>&1 && echo single ok
