set -o pipefail
mkdir -p gpurun_out/r6b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b
timeout -k 10 300 python benchmarks/gemm_sweep.py --cfgs 12,2,3,24,25 --cases fwd1,fwd2,dgrad2 --out $O/sweep.json > $O/sweep.log 2>&1 && echo sweep ok &&
timeout -k 10 120 python benchmarks/pair_stamps.py --out $O/pair_stamps.json > $O/pair_stamps.log 2>&1 && echo stamps ok &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_layouts and (24 or 25)" > $O/t_gemm.log 2>&1 && echo tgemm ok &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_deepnn.py > $O/t_deepnn.log 2>&1 && echo tdeepnn ok &&
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > $O/deepnn.log 2>&1 && echo bdeepnn ok &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_f32.py > $O/tests.log 2>&1 && echo tests ok
