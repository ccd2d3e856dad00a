set -o pipefail
mkdir -p gpurun_out/r5ad
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ad/smoke.log 2>&1
echo smoke rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ad/b20_1.log 2>&1
echo b1 rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ad/b20_2.log 2>&1
echo b2 rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/r5ad/b200.log 2>&1
echo b3 rc=$?
timeout -k 10 300 python bench.py > gpurun_out/r5ad/bdefault.log 2>&1
echo b4 rc=$?
