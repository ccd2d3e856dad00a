set -o pipefail
mkdir -p gpurun_out/r5i
for i in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5i/between_$i.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --stock_between 0 > gpurun_out/r5i/after_$i.json 2>/dev/null || exit 1
done
echo ab rc=$?
