set -o pipefail
mkdir -p gpurun_out/r5bq
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bq/gpu_suite.log 2>&1
echo suite rc=$?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5bq/smoke.log 2>&1
echo smoke rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5bq/b20.log 2>&1
echo b20 rc=$?
timeout -k 10 300 python bench.py > gpurun_out/r5bq/bdefault.log 2>&1
echo bdef rc=$?
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > gpurun_out/r5bq/vgg32.log 2>&1
echo v32 rc=$?
