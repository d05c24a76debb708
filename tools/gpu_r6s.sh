#!/bin/bash
# PTB world-1: LocalOptimizer vs DistriOptimizer host profile (cumulative)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s
mkdir -p $O
for arm in local distri; do
  f=""; [ $arm = distri ] && f="--force-distri"
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --cprofile 100 $f > $O/cp_$arm.log 2>&1 || { tail -20 $O/cp_$arm.log; exit 1; }
  grep '^{' $O/cp_$arm.log | cut -c1-160
  grep "function calls" $O/cp_$arm.log
done
