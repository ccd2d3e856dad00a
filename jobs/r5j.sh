set -o pipefail
mkdir -p gpurun_out/r5j
for i in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5j/warm_$i.json 2>/dev/null || exit 1
DDPX_GRAPH_COLD_OK=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5j/cold_$i.json 2>/dev/null || exit 1
done
echo ab rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/r5j/b200.json 2>/dev/null
echo rc=$?
