set -o pipefail
mkdir -p gpurun_out/r5bc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
for pr in 0 1; do
DDPX_GEMM_PRIO=$pr timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 --stock_ref 0 > gpurun_out/r5bc/vgg_${pr}_$i.log 2>&1
echo b $pr $i rc=$?
done
done
DDPX_GEMM_PRIO=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bc/p1 -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bc/prof1.log 2>&1
echo p1 rc=$?
DDPX_GEMM_PRIO=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5bc/p0 -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5bc/prof0.log 2>&1
echo p0 rc=$?
