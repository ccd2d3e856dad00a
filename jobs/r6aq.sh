set -o pipefail
O=gpurun_out/r6aq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python benchmarks/f32_first_conv_probe.py > $O/probe_ring3.jsonl 2>$O/probe_ring3.err || exit 1
DDPX_F32_SMALLK=0 timeout -k 10 200 python benchmarks/f32_first_conv_probe.py > $O/probe_ring4.jsonl 2>$O/probe_ring4.err || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 --stock_ref 0 > $O/d32_ring3.json 2>$O/d32_ring3.err || exit 1
DDPX_F32_SMALLK=0 timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 --stock_ref 0 > $O/d32_ring4.json 2>$O/d32_ring4.err || exit 1
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/v32_ring3.json 2>$O/v32_ring3.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py -q -x --timeout 200 --timeout-method thread > $O/f32_tests.log 2>&1 || exit 1
echo done
