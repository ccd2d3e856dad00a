set -o pipefail
mkdir -p gpurun_out/r5ao
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vgg.py tests/test_gpu_deepnn.py > gpurun_out/r5ao/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ao/vgg_1.log 2>&1
echo n1 rc=$?
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > gpurun_out/r5ao/deepnn_1.log 2>&1
echo d1 rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ao/vgg_2.log 2>&1
echo n2 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ao/new -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ao/prof.log 2>&1
echo p1 rc=$?
