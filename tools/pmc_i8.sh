#!/bin/bash
# PMC passes (kernel-trace only) on the short-reduction int8 convs: 64→256 1x1 at 56² with the int8
# residual (tile v0) and 256→64 1x1 at 56² (the non-short-K 256x64 tile), batch 256
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/pmci8
mkdir -p $R
i=0
for spec in "64,256,56,1 0" "64,256,56,0 0" "256,64,56,0 0"; do
  set -- $spec
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/p$i -o run -- python3 tools/i8_shortk_bench.py $1 $2 > $R/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/p$i.log; exit 1; }
    echo "$i $1:v$2 $grp" >> $R/index.txt
  done
done
find $R -name "*.db" -delete
python3 tools/pmc_summary.py $R k_conv_i8 > $R/summary.txt 2>&1 || true
cat $R/summary.txt | head -60
