set -o pipefail
mkdir -p gpurun_out/r5az
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_deepnn.py > gpurun_out/r5az/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > gpurun_out/r5az/deepnn.log 2>&1
echo b1 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5az/deepnn -o dn -- python bench.py --model deepnn --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5az/dn.log 2>&1
echo p1 rc=$?
