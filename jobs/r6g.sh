set -o pipefail
mkdir -p gpurun_out/r6g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad_sgd_pair_matches" > $O/t_pair.log 2>&1 && echo tpair ok &&
timeout -k 10 60 python benchmarks/pair_stamps.py --time_only > $O/xwg_time.log 2>&1 && echo xwg ok &&
DDPX_WSGD_XWG=0 timeout -k 10 60 python benchmarks/pair_stamps.py --time_only > $O/ws_time.log 2>&1 && echo ws ok &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b200.log 2>&1 && echo b200 ok &&
DDPX_WSGD_XWG=0 timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b200_ws.log 2>&1 && echo b200ws ok
