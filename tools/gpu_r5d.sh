#!/bin/bash
# PMC passes on the fp32 direct conv kernels (conv_x3): a pointwise and a 3x3 shape
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/pmc5; mkdir -p gpurun_out/pmc5
i=0
for spec in "256,1024,1,1,14 fwd" "128,128,3,1,28 fwd" "64,256,1,1,56 fwd"; do
  set -- $spec
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc5/p$i -o run -- python3 tools/conv_one.py --f32 --shape $1 --op $2 --iters 10 > gpurun_out/pmc5/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc5/p$i.log; exit 1; }
    echo "$i $1:$2 $grp" >> gpurun_out/pmc5/index.txt
  done
done
find gpurun_out/pmc5 -name "*.db" -delete
python3 tools/pmc_summary.py gpurun_out/pmc5 > gpurun_out/pmc5/summary.txt 2>&1; cat gpurun_out/pmc5/summary.txt
