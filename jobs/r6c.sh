set -o pipefail
mkdir -p gpurun_out/r6c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c
timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair_x0.json > $O/pair_x0.log 2>&1 && echo x0 ok &&
DDPX_WSGD_XTRA=3 timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair_x3.json > $O/pair_x3.log 2>&1 && echo x3 ok &&
DDPX_WSGD_XTRA=4 timeout -k 10 120 python benchmarks/pair_stamps.py --reps 3 --out $O/pair_x4.json > $O/pair_x4.log 2>&1 && echo x4 ok &&
timeout -k 10 300 python benchmarks/gemm_sweep.py --cfgs 12,3,5,7,1,21,13,14 --cases wgrad2,wgrad2kk --out $O/sweep_wgrad.json > $O/sweep_wgrad.log 2>&1 && echo sweep ok &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_deepnn.py > $O/t_deepnn.log 2>&1 && echo tdeepnn ok &&
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > $O/deepnn.log 2>&1 && echo bdeepnn ok &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_f32.py > $O/tests.log 2>&1 && echo tests ok
