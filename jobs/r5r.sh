set -o pipefail
mkdir -p gpurun_out/r5r
timeout -k 10 300 python benchmarks/wino_bench.py --out gpurun_out/r5r/wino3.json > gpurun_out/r5r/wino3.txt 2>&1
echo b3 rc=$?
DDPX_WINO_STAGES=2 timeout -k 10 300 python benchmarks/wino_bench.py --out gpurun_out/r5r/wino2.json > gpurun_out/r5r/wino2.txt 2>&1
echo b2 rc=$?
