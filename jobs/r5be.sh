set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/wp/a -- python3 $R/benchmarks/wino_probe.py > $R/gpurun_out/wp_a.log 2>&1 || exit 3
echo a ok
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/wp/b -- python3 $R/benchmarks/wino_probe.py > $R/gpurun_out/wp_b.log 2>&1 || exit 3
echo b ok
