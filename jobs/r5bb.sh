set -o pipefail
mkdir -p gpurun_out/r5bb
for pr in 0 1; do
DDPX_GEMM_PRIO=$pr timeout -k 10 400 python benchmarks/conv_sweep.py --cfgs 13,22,23 --layers 1,3,5 --out gpurun_out/r5bb/sweep_$pr.json > gpurun_out/r5bb/sweep_$pr.log 2>&1
echo sweep $pr rc=$?
done
DDPX_GEMM_PRIO=1 timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5bb/vgg_1.log 2>&1
echo b1 rc=$?
DDPX_GEMM_PRIO=0 timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > gpurun_out/r5bb/vgg_0.log 2>&1
echo b0 rc=$?
