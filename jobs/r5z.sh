set -o pipefail
mkdir -p gpurun_out/r5z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --dtype fp32 --steps 100 --warmup 10 --stock_ref 1 > gpurun_out/r5z/mlp32.log 2>&1
echo b rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5z/prof -o mlp32 -- python bench.py --dtype fp32 --steps 30 --warmup 5 --stock_ref 0 > gpurun_out/r5z/prof.log 2>&1
echo prof rc=$?
