set -o pipefail
mkdir -p gpurun_out/r6h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h
DDPX_WSGD_XWG_LOCAL=1 timeout -k 10 60 python benchmarks/pair_stamps.py --xwg > $O/xwg_local.log 2>&1 && echo local ok &&
DDPX_WSGD_XTRA=3 DDPX_WSGD_XWG=0 timeout -k 10 60 python benchmarks/pair_stamps.py --time_only > $O/ws_x3.log 2>&1 && echo x3 ok &&
DDPX_WSGD_XTRA=4 DDPX_WSGD_XWG=0 timeout -k 10 60 python benchmarks/pair_stamps.py --time_only > $O/ws_x4.log 2>&1 && echo x4 ok
