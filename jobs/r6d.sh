set -o pipefail
mkdir -p gpurun_out/r6d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d
export DDPX_WSGD_XTRA=3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $O/x3/a -o a -- python benchmarks/pair_stamps.py --reps 1 > $O/x3_a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TA_TA_BUSY TCP_TCC_READ_REQ GRBM_GUI_ACTIVE --output-format csv -d $O/x3/b -o b -- python benchmarks/pair_stamps.py --reps 1 > $O/x3_b.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/x3/c -o c -- python benchmarks/pair_stamps.py --reps 1 > $O/x3_c.log 2>&1 && echo pmc ok &&
unset DDPX_WSGD_XTRA &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_deepnn.py > $O/t_deepnn.log 2>&1 && echo tdeepnn ok &&
timeout -k 10 300 python bench.py --model deepnn --steps 30 --warmup 5 > $O/deepnn.log 2>&1 && echo bdeepnn ok &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_f32.py > $O/tests.log 2>&1 && echo tests ok
