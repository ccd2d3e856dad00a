set -o pipefail
O=gpurun_out/r6at
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py -q -x --timeout 200 --timeout-method thread > $O/f32_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32.json 2>$O/d32.err || exit 1
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 > $O/v32.json 2>$O/v32.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pd -o d32 -- python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/pd.log 2>&1 || exit 1
echo done
