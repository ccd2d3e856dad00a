set -o pipefail
O=gpurun_out/r6au
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_deepnn.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32_pad.json 2>$O/d32_pad.err || exit 1
DDPX_F32_WINO_WGRAD_PAD=0 timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32_nopad.json 2>$O/d32_nopad.err || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/d32_pad2.json 2>$O/d32_pad2.err || exit 1
echo done
