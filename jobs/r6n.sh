set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
DDPX_WINO_STAGES=3 timeout -k 10 200 python benchmarks/wino_bench.py --out $O/layers_s3.json > $O/layers_s3.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pa -- python3 $R/benchmarks/wino_probe.py > $O/pa.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d $R/$O/pb -- python3 $R/benchmarks/wino_probe.py > $O/pb.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $R/$O/pc -- python3 $R/benchmarks/wino_probe.py > $O/pc.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p -o v32 -- python bench.py --model vgg --dtype fp32 --steps 6 --warmup 2 --stock_ref 0 > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8.log 2>&1 || exit 1
DDPX_WSGD_MATH_WAVES=4 timeout -k 10 300 python bench.py --model mlp_wide --fp8 1 --steps 20 --warmup 5 --stock_ref 0 > $O/wide_fp8_mw4.log 2>&1 || exit 1
DDPX_WSGD_MATH_WAVES=4 timeout -k 10 300 python bench.py --model mlp_wide --steps 20 --warmup 5 --stock_ref 0 > $O/wide_mw4.log 2>&1 || exit 1
echo done
