#!/bin/bash
# PMC counters for the conv kernels on two representative ResNet-50 shapes (separate passes,
# kernel-trace only — no sys/runtime trace with --pmc on this pool).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for shape in 256,256,3,1,14 1024,256,1,1,14 64,256,1,1,56; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/conv_one.py --shape $shape --iters 10 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
    echo "$i $shape $grp" >> gpurun_out/pmc/index.txt
  done
done
echo pmc done
find gpurun_out/pmc -name "*.db" -delete
du -sh gpurun_out/pmc
