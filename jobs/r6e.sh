set -o pipefail
mkdir -p gpurun_out/r6e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e
timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair8_x0.json > $O/pair8_x0.log 2>&1 && echo x0 ok &&
DDPX_WSGD_XTRA=3 timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair8_x3.json > $O/pair8_x3.log 2>&1 && echo x3 ok &&
DDPX_WSGD_MATH_WAVES=4 timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair4_x0.json > $O/pair4_x0.log 2>&1 && echo x0_4 ok &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad_sgd" tests/test_gpu_fp8.py > $O/t_pair.log 2>&1 && echo tpair ok &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b200.log 2>&1 && echo b200 ok &&
DDPX_WSGD_MATH_WAVES=4 timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b200_mw4.log 2>&1 && echo b200mw4 ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mlp -o mlp -- python bench.py --steps 30 --warmup 5 --stock_ref 0 > $O/prof_mlp.log 2>&1 && echo p2 ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/deepnn -o deepnn -- python bench.py --model deepnn --steps 20 --warmup 3 --stock_ref 0 > $O/prof_deepnn.log 2>&1 && echo p1 ok &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_dist.py -k side_stream > $O/t_side.log 2>&1 && echo tside ok
