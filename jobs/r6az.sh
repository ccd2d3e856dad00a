set -o pipefail
O=gpurun_out/r6az
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20.json 2>$O/b20.err || exit 1
timeout -k 10 300 python bench.py --model vgg --dtype fp32 --steps 20 --warmup 3 > $O/vgg32.json 2>$O/vgg32.err || exit 1
timeout -k 10 300 python bench.py --model vgg --steps 20 --warmup 3 > $O/vgg.json 2>$O/vgg.err || exit 1
timeout -k 10 300 python bench.py --model deepnn --steps 40 --warmup 5 > $O/deepnn.json 2>$O/deepnn.err || exit 1
timeout -k 10 300 python bench.py --dtype fp32 --steps 200 --warmup 10 > $O/mlp32.json 2>$O/mlp32.err || exit 1
echo done
