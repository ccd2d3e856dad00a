set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python benchmarks/gemm_sweep.py --hidden 16384 --cases fwd1,fwd2,dgrad2 --cfgs 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25 --iters 20 --out $O/wide_sweep.json > $O/wide_sweep.log 2>&1 || exit 1
echo done
