#!/bin/bash
# PMC counters (separate passes, kernel-trace only) for the three conv kernel regimes of the
# ResNet-50 step: expand 1x1 (BK=32), stage-1 1x1 (memory-bound), 3x3 (BK=64).  Args: op list.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
i=0
IFS=';' read -ra LIST <<< "${SPECS:-256,1024,1,1,14 fwdstats;64,256,1,1,56 fwdstats;128,128,3,1,28 fwdstats;256,1024,1,1,14 dgrad}"
for spec in "${LIST[@]}"; do
  set -- $spec
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc2/p$i -o run -- python3 tools/conv_one.py --shape $1 --op $2 --iters 10 > gpurun_out/pmc2/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc2/p$i.log; exit 1; }
    echo "$i $1:$2 $grp" >> gpurun_out/pmc2/index.txt
  done
done
echo pmc done
find gpurun_out/pmc2 -name "*.db" -delete
