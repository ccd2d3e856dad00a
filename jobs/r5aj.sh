set -o pipefail
mkdir -p gpurun_out/r5aj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vgg.py tests/test_gpu_deepnn.py tests/test_gpu_parity.py > gpurun_out/r5aj/tests.log 2>&1
echo tests rc=$?
for i in 1 2; do
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5aj/vgg_new_$i.log 2>&1
echo n$i rc=$?
DDPX_CONV_PICKS=r4 DDPX_BN_MERGE=bwd timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5aj/vgg_r4_$i.log 2>&1
echo r$i rc=$?
done
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > gpurun_out/r5aj/deepnn_new.log 2>&1
echo d rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5aj/new -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5aj/prof.log 2>&1
echo p1 rc=$?
