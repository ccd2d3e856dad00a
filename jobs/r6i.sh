set -o pipefail
mkdir -p gpurun_out/r6i
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
export DDPX_WSGD_XWG=0
for x in 0 3 4; do
DDPX_WSGD_XTRA=$x timeout -s KILL 90 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ TA_TA_BUSY TCP_TCC_READ_REQ GRBM_GUI_ACTIVE --output-format csv -d $O/x$x -o p -- python benchmarks/pair_stamps.py --time_only > $O/x$x.log 2>&1 || exit 1
done; echo pmc ok
