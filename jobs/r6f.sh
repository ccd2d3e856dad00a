set -o pipefail
mkdir -p gpurun_out/r6f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f
DDPX_WSGD_STAGES=4 timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair8_s4.json > $O/pair8_s4.log 2>&1 && echo s4 ok &&
DDPX_WSGD_STAGES=4 DDPX_WSGD_XTRA=3 timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 > $O/pair8_s4_x3.log 2>&1 && echo s4x3 ok &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_deepnn.py tests/test_gpu_kernels.py > $O/t.log 2>&1 && echo t ok &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b200.log 2>&1 && echo b200 ok &&
DDPX_WSGD_STAGES=4 timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b200_s4.log 2>&1 && echo b200s4 ok &&
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > $O/deepnn.log 2>&1 && echo bdeepnn ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/deepnn -o deepnn -- python bench.py --model deepnn --steps 20 --warmup 3 --stock_ref 0 > $O/prof_deepnn.log 2>&1 && echo p1 ok
