set -o pipefail
O=gpurun_out/r6am
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -m gpu -q --timeout 300 --timeout-method thread -k "deepnn or bias or relu or pool" > $O/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/t.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --model deepnn --dtype fp32 --steps 20 --warmup 3 --stock_ref 1 --stock_steps 10 > $O/deepnn32.log 2>&1 || exit 1
echo done
