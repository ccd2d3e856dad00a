set -o pipefail
mkdir -p gpurun_out/r5p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/r5p/tests_f32.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5p/vgg32_stock.log 2>&1
echo bench rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5p/prof -o run -- python bench.py --model vgg --dtype fp32 --steps 5 --warmup 2 --stock_ref 0 > gpurun_out/r5p/prof.log 2>&1
echo prof rc=$?
