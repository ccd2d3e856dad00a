set -o pipefail
mkdir -p gpurun_out/r5u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 --stock_ref 1 --stock_steps 10 > gpurun_out/r5u/vgg_bf16.log 2>&1
echo bench rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5u/prof -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > gpurun_out/r5u/prof.log 2>&1
echo prof rc=$?
