set -o pipefail
O=gpurun_out/r6ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ok() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1; ok $? b20 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/b200.log 2>&1; ok $? b200 || exit 1
timeout -k 10 300 python bench.py --model vgg --steps 30 --warmup 5 > $O/vgg.log 2>&1; ok $? vgg || exit 1
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > $O/vgg32.log 2>&1; ok $? vgg32 || exit 1
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > $O/deepnn.log 2>&1; ok $? deepnn || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > $O/deepnn32.log 2>&1; ok $? deepnn32 || exit 1
timeout -k 10 300 python bench.py --dtype fp32 --steps 100 --warmup 10 --stock_ref 1 > $O/mlp32.log 2>&1; ok $? mlp32 || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --steps 20 --warmup 5 > $O/wide.log 2>&1; ok $? wide || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8.log 2>&1; ok $? wide_fp8 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --ddp_single --sim_world 8 --shard_optimizer 1 --bucket_plan default --steps 200 --warmup 20 --stock_ref 0 > $O/sim8_zero1.log 2>&1; ok $? sim8 || exit 1
echo done
