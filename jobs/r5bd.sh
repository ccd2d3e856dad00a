set -o pipefail
mkdir -p gpurun_out/r5bd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vgg.py -k "merge or bn or native" > gpurun_out/r5bd/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bd/p -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bd/prof.log 2>&1
echo p1 rc=$?
