set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
DDPX_FP8_DGRAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pd -o w8d -- python bench.py --model mlp_wide --fp8 1 --steps 10 --warmup 3 --stock_ref 0 > $O/pd.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p8 -o w8 -- python bench.py --model mlp_wide --fp8 1 --steps 10 --warmup 3 --stock_ref 0 > $O/p8.log 2>&1 || exit 1
echo done
