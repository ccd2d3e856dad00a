set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_deepnn.py tests/test_gpu_kernels.py tests/test_gpu_fp8.py -m gpu -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/t.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > $O/deepnn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --stock_ref 0 > $O/toy.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pd -o dn -- python bench.py --model deepnn --steps 20 --warmup 3 --stock_ref 0 > $O/pd.log 2>&1 || exit 1
echo done
