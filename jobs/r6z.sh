set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fp8.py -m gpu -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/t.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --steps 20 --warmup 5 > $O/wide.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8.log 2>&1 || exit 1
DDPX_FP8_DGRAD=1 timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8_dgrad.log 2>&1 || exit 1
echo done
