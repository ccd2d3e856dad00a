set -o pipefail
mkdir -p gpurun_out/r6k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_suite.log 2>&1; echo suite rc=$?
