set -o pipefail
mkdir -p gpurun_out/r5ai
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ai/new -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ai/new.log 2>&1
echo p1 rc=$?
DDPX_CONV_PICKS=r4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ai/r4 -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ai/r4.log 2>&1
echo p2 rc=$?
