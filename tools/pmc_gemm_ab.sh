set -e
o=gpurun_out/p3; mkdir -p $o
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum"
for arm in cfg9 lib; do
  extra="--cfg 9"; [ $arm = lib ] && extra="--library"
  timeout -s KILL 90 rocprofv3 --pmc $A -d $o/${arm}_a -o run --output-format csv -- python3 tools/prof_gemm_one.py --shape gate_up --M 8192 --iters 5 $extra > $o/${arm}_a.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $B -d $o/${arm}_b -o run --output-format csv -- python3 tools/prof_gemm_one.py --shape gate_up --M 8192 --iters 5 $extra > $o/${arm}_b.log 2>&1
done
