set -o pipefail
mkdir -p gpurun_out/r5v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in wino_fwd_h8 wgrad_h8 wino_fwd_h32 wgrad_h32; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r5v/a_$c -o p -- python3 benchmarks/f32_probe.py --case $c > gpurun_out/r5v/a_$c.log 2>&1 || { echo "pass a $c failed"; exit 1; }
  echo a $c ok
done
for c in wino_fwd_h8 wgrad_h8; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM --output-format csv -d gpurun_out/r5v/b_$c -o p -- python3 benchmarks/f32_probe.py --case $c > gpurun_out/r5v/b_$c.log 2>&1 || { echo "pass b $c failed"; exit 1; }
  echo b $c ok
done
