set -o pipefail
O=gpurun_out/r6as
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python benchmarks/conv_sweep.py --layers 2,3,4,5,6 --cfgs 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,21,22,23 --out $O/sweep.json > $O/sweep.log 2>&1 || exit 1
echo done
