set -o pipefail
O=gpurun_out/r6ar
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pv -o vgg -- python bench.py --model vgg --steps 20 --warmup 3 --stock_ref 0 > $O/pv.log 2>&1 || exit 1
echo done
