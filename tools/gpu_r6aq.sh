#!/bin/bash
# round-6 end evidence: step HBM bytes (bf16), PMC of the 56² 64→256 data gradient and the 3x3 / deep 1x1 forwards,
# every BASELINE config x3 (bench_configs), int8 pair path (ResNet-50 x3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aq
mkdir -p $O
bash tools/pmc_step_bytes.sh > $O/step_bytes.log 2>&1 || { tail -20 $O/step_bytes.log; exit 1; }
cp gpurun_out/pmcstep/summary.txt $O/step_bytes_summary.txt
head -3 $O/step_bytes_summary.txt
SPECS="64,256,1,1,56 dgrad;64,256,1,1,56 fwdstats;128,128,3,1,28 fwdstats;1024,256,1,1,14 fwdstats" bash tools/pmc_conv2.sh > $O/pmc_conv.log 2>&1 || { tail -20 $O/pmc_conv.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc2 > $O/pmc_conv_summary.txt 2>&1 || true
grep -E "==|MFMA util|VALU per|L2 hit|median" $O/pmc_conv_summary.txt | head -40
for i in 1 2 3; do
  for c in vgg inception ptb transformer lenet; do
    timeout -k 10 300 python tools/bench_configs.py --config $c --steps 20 --warmup 5 > $O/cfg_${c}_$i.log 2>&1 || { tail -20 $O/cfg_${c}_$i.log; exit 1; }
    grep '^{' $O/cfg_${c}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"][:60], d["value"], d["ms_per_step"], d.get("dtype"))'
  done
done
