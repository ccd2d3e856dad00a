set -o pipefail
mkdir -p gpurun_out/r5av
for sl in 1024 1536 768; do
DDPX_WINO_WGRAD_SLOTS=$sl timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f32.py -k "wino_wgrad" > gpurun_out/r5av/tests_$sl.log 2>&1
echo tests $sl rc=$?
DDPX_WINO_WGRAD_SLOTS=$sl timeout -k 10 200 python benchmarks/wino_bench.py --only wgrad --out gpurun_out/r5av/wgrad_$sl.json > gpurun_out/r5av/wgrad_$sl.log 2>&1
echo bench $sl rc=$?
done
