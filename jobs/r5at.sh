set -o pipefail
mkdir -p gpurun_out/r5at
for v in s2w0 s2w1 s3w0 s3w1; do
DDPX_WINO_WGRAD_VARIANT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f32.py -k "wino_wgrad" > gpurun_out/r5at/tests_$v.log 2>&1
echo tests $v rc=$?
DDPX_WINO_WGRAD_VARIANT=$v timeout -k 10 200 python benchmarks/wino_bench.py --only wgrad --out gpurun_out/r5at/wgrad_$v.json > gpurun_out/r5at/wgrad_$v.log 2>&1
echo bench $v rc=$?
done
