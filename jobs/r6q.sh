set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "8 8" "8 4" "4 4" "4 8"; do set -- $cfg
DDPX_WSGD_STREAM_WAVES=$1 DDPX_WSGD_MATH_WAVES=$2 timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/fp8_sw$1_mw$2.log 2>&1 || exit 1
done
DDPX_WSGD_STREAM_WAVES=8 timeout -k 10 300 python bench.py --model mlp_wide --steps 20 --warmup 5 --stock_ref 0 > $O/bf16_sw8.log 2>&1 || exit 1
echo done
