set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_entrypoints.py tests/test_gpu_multirank.py -m gpu -q -k "wino or vgg or sync_batchnorm or reference_command or without_nprocs" --timeout 120 --timeout-method thread > $O/t_wino.log 2>&1; rc=$?; echo t_wino rc=$rc; tail -3 $O/t_wino.log; [ $rc -le 1 ] || exit 1
timeout -k 10 200 python benchmarks/wino_bench.py --out $O/layers_asm.json > $O/layers_asm.log 2>&1 || exit 1
DDPX_WINO_STAGES=2c timeout -k 10 200 python benchmarks/wino_bench.py --out $O/layers_2c.json > $O/layers_2c.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/vgg32.log 2>&1 || exit 1
DDPX_WINO_STAGES=2c timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/vgg32_2c.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/deepnn32.log 2>&1 || exit 1
echo done
