set -o pipefail
O=gpurun_out/r6af
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -m gpu -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/t.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --steps 20 --warmup 5 --stock_ref 0 > $O/wide.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8_2.log 2>&1 || exit 1
echo done
