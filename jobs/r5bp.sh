set -o pipefail
mkdir -p gpurun_out/r5bp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/r5bp/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bp/p -o v32 -- python bench.py --model vgg --dtype fp32 --steps 6 --warmup 2 --stock_ref 0 > gpurun_out/r5bp/prof.log 2>&1
echo p1 rc=$?
