set -o pipefail
mkdir -p gpurun_out/r5ax
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vgg.py > gpurun_out/r5ax/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ax/vgg_1.log 2>&1
echo b1 rc=$?
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5ax/vgg_2.log 2>&1
echo b2 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ax/new -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ax/prof.log 2>&1
echo p1 rc=$?
