#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6d
SYNC=0 STEPS=14 timeout -k 10 300 python tools/fp32_steps.py > gpurun_out/r6d/nosync.log 2>&1 || { tail -20 gpurun_out/r6d/nosync.log; exit 1; }
grep "^step\|final" gpurun_out/r6d/nosync.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 10 > gpurun_out/r6d/b_$i.log 2>&1 || { tail -20 gpurun_out/r6d/b_$i.log; exit 1; }
  grep metric gpurun_out/r6d/b_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bf16", d["ms_per_step"], d["value"], "fp32", d["fp32"])'
done
