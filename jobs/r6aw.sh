set -o pipefail
O=gpurun_out/r6aw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/f32_first_wgrad_probe.py > $O/probe.jsonl 2>$O/probe.err || exit 1
echo done
