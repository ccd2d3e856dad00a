set -o pipefail
O=gpurun_out/r6ax
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_deepnn.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32_mask.json 2>$O/d32_mask.err || exit 1
DDPX_F32_DGRAD_MASK=0 timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32_nomask.json 2>$O/d32_nomask.err || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32_mask2.json 2>$O/d32_mask2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pd -o d32 -- python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/pd.log 2>&1 || exit 1
echo done
