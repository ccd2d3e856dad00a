set -o pipefail
mkdir -p gpurun_out/r5h
for i in 1 2; do
DDPX_STEP_TRACE=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --stock_ref 0 > gpurun_out/r5h/trace_$i.json 2> gpurun_out/r5h/trace_$i.err || exit 1
done
DDPX_STEP_TRACE=1 timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --stock_ref 0 > gpurun_out/r5h/trace60.json 2> gpurun_out/r5h/trace60.err
echo rc=$?
