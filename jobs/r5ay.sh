set -o pipefail
mkdir -p gpurun_out/r5ay
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ay/deepnn -o dn -- python bench.py --model deepnn --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5ay/dn.log 2>&1
echo p1 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ay/vgg32 -o v32 -- python bench.py --model vgg --dtype fp32 --steps 6 --warmup 2 --stock_ref 0 > gpurun_out/r5ay/v32.log 2>&1
echo p2 rc=$?
