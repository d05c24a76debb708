#!/bin/bash
# int8 ResNet-50 / Inception forward: per-launch trace of the last forward passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ae
mkdir -p $O
for mdl in resnet50 inception; do
  timeout -k 10 600 rocprofv3 --kernel-trace -d $O/p_$mdl -o run -- python3 tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 4 --warmup 2 > $O/p_$mdl.log 2>&1 || { tail -20 $O/p_$mdl.log; exit 1; }
  db=$(find $O/p_$mdl -name '*.db' | head -1)
  python3 tools/rocpd_dispatches.py "$db" 900 > $O/d_$mdl.txt
  rm -rf $O/p_$mdl
done
echo done
