set -o pipefail
O=gpurun_out/r6al
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pm -o m32 -- python bench.py --dtype fp32 --steps 40 --warmup 5 --stock_ref 0 > $O/pm.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pd -o d32 -- python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/pd.log 2>&1 || exit 1
echo done
