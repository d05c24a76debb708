#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
for i in 1 2 3; do
  SYNC=0 STEPS=14 timeout -k 10 300 python tools/fp32_steps.py > gpurun_out/r6c/nosync_$i.log 2>&1 || { tail -20 gpurun_out/r6c/nosync_$i.log; exit 1; }
  grep "^step\|final" gpurun_out/r6c/nosync_$i.log
done
