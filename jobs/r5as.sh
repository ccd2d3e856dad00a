set -o pipefail
mkdir -p gpurun_out/r5as
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5as/prof -o vgg32 -- python bench.py --model vgg --dtype fp32 --steps 6 --warmup 2 --stock_ref 0 > gpurun_out/r5as/prof.log 2>&1
echo p1 rc=$?
