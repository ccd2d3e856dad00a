set -o pipefail
mkdir -p gpurun_out/r5ba
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "augment" tests/test_gpu_f32.py::test_augment_nhwc4_f32_matches_cpu tests/test_gpu_entrypoints.py > gpurun_out/r5ba/tests.log 2>&1
echo tests rc=$?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/r5ba/b200.log 2>&1
echo b1 rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5ba/b20.log 2>&1
echo b2 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ba/mlp -o mlp -- python bench.py --steps 40 --warmup 5 --stock_ref 0 > gpurun_out/r5ba/prof.log 2>&1
echo p1 rc=$?
