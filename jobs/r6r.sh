set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cp in 0 1 2; do
DDPX_WSGD_CACHE=$cp timeout -k 10 120 python benchmarks/pair_stamps.py --time_only > $O/pair_cp$cp.log 2>&1 || exit 1
done
for cp in 0 1 2 0 1 2; do
DDPX_WSGD_CACHE=$cp timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --stock_ref 0 >> $O/bench_cp$cp.log 2>&1 || exit 1
done
echo done
