set -o pipefail
mkdir -p gpurun_out/r5e
timeout -k 10 300 python benchmarks/gemm_stamps.py --out gpurun_out/r5e/stamps.json > gpurun_out/r5e/stamps.txt 2>&1
echo stamps rc=$?
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread "tests/test_gpu_multirank.py::test_native_sync_batchnorm_two_ranks_one_gpu" > gpurun_out/r5e/syncbn.log 2>&1
echo syncbn rc=$?
