set -o pipefail
O=gpurun_out/r6ak
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_entrypoints.py -m gpu -q --timeout 300 --timeout-method thread -k "bench" > $O/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -5 $O/t.log
