#!/bin/bash
# ResNet-50 bf16 vs fp32 training curves on the learnable synthetic task (tools/convergence.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ag
mkdir -p $O
for dt in bf16 fp32; do
  timeout -k 10 500 python -u tools/convergence.py --dtype $dt --steps 1500 --batch 128 --log-every 50 > $O/conv_$dt.log 2>&1 || { tail -20 $O/conv_$dt.log; exit 1; }
  grep '^{' $O/conv_$dt.log | tail -3
done
