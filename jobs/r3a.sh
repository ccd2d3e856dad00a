set -o pipefail
mkdir -p gpurun_out/r3a
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench20.json 2> gpurun_out/r3a/bench20.err &&
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 > gpurun_out/r3a/bench100.json 2> gpurun_out/r3a/bench100.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a/prof -o mlp -- python bench.py --gpus 1 --steps 50 --warmup 5 --stock_ref 0 > gpurun_out/r3a/prof.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --model vgg --steps 20 --warmup 5 > gpurun_out/r3a/vgg.json 2> gpurun_out/r3a/vgg.err &&
timeout -k 10 300 python bench.py --gpus 1 --model mlp_wide --steps 20 --warmup 5 > gpurun_out/r3a/wide.json 2> gpurun_out/r3a/wide.err &&
timeout -k 10 300 python bench.py --gpus 1 --model mlp_wide --fp8 1 --steps 20 --warmup 5 > gpurun_out/r3a/wide_fp8.json 2> gpurun_out/r3a/wide_fp8.err
