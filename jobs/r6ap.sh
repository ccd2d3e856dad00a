set -o pipefail
O=gpurun_out/r6ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python benchmarks/f32_first_conv_probe.py > $O/probe_vec.jsonl 2>$O/probe_vec.err || exit 1
DDPX_F32_EPI=scalar timeout -k 10 200 python benchmarks/f32_first_conv_probe.py > $O/probe_scalar.jsonl 2>$O/probe_scalar.err || exit 1
echo done
