set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fp8.py tests/test_gpu_dist.py -m gpu -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/t.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pt -o toy -- python bench.py --gpus 1 --steps 40 --warmup 5 --stock_ref 0 > $O/pt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pw -o wide -- python bench.py --model mlp_wide --steps 10 --warmup 3 --stock_ref 0 > $O/pw.log 2>&1 || exit 1
echo done
