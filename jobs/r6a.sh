set -o pipefail
mkdir -p gpurun_out/r6a
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 && echo bench ok &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_entrypoints.py -k "n_gt_1 or survives or contract" tests/test_gpu_dist.py > $O/tests1.log 2>&1 && echo tests1 ok &&
for c in fwd0_t-1 fwd1_t-1 dgrad1_t-1; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$c/a -o a -- python benchmarks/kernel_probe.py --case $c > $O/pmc_${c}_a.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TA_TA_BUSY TCP_TCC_READ_REQ GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$c/b -o b -- python benchmarks/kernel_probe.py --case $c > $O/pmc_${c}_b.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$c/c -o c -- python benchmarks/kernel_probe.py --case $c > $O/pmc_${c}_c.log 2>&1 || exit 1
done && echo pmc ok
