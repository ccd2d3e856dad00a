set -o pipefail
mkdir -p gpurun_out/r5bi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DDPX_WG_SPLIT4=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bi/s1 -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bi/s1.log 2>&1
echo p1 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bi/s2 -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bi/s2.log 2>&1
echo p2 rc=$?
