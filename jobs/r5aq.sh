set -o pipefail
mkdir -p gpurun_out/r5aq
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f32.py -k "wino_wgrad or wino or fp32" > gpurun_out/r5aq/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python benchmarks/wino_bench.py --out gpurun_out/r5aq/layers.json > gpurun_out/r5aq/layers.log 2>&1
echo bench rc=$?
