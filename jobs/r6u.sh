set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python benchmarks/pair_fp8t.py > $O/pair_fp8t.log 2>&1 || exit 1
echo done
