set -o pipefail
O=gpurun_out/r6ay
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
ok() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 200 python benchmarks/f32_first_conv_probe.py > $O/probe_final.jsonl 2>$O/probe_final.err; ok $? probe || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 40 --warmup 5 > $O/final_deepnn32.json 2>$O/d32.err; ok $? d32 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_suite.log 2>&1; ok $? suite || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; ok $? smoke || exit 1
timeout -k 10 300 python bench.py > $O/bdefault.log 2>&1; ok $? bdefault || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pd -o d32 -- python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 0 > $O/pd.log 2>&1; ok $? prof || exit 1
echo done
