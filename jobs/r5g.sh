set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 300 python benchmarks/window_probe.py --out gpurun_out/r5g/window.json > gpurun_out/r5g/window.txt 2>&1
echo window rc=$?
for i in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5g/warm_$i.json 2>/dev/null || exit 1
DDPX_GRAPH_COLD_OK=1 DDPX_GRAPH_SIZES=1,20 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5g/cold_$i.json 2>/dev/null || exit 1
done
echo ab rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/r5g/b200.json 2>/dev/null
echo b200 rc=$?
