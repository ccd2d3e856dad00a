set -o pipefail
mkdir -p gpurun_out/r5bm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vgg.py tests/test_gpu_deepnn.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_kernels.py > gpurun_out/r5bm/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5bm/vgg.log 2>&1
echo b1 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bm/p -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bm/prof.log 2>&1
echo p1 rc=$?
