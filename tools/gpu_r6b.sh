#!/bin/bash
# round 6: fp32 repeat stability (outlier hunt) + bf16 headline check
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > gpurun_out/r6b/f32_$i.log 2>&1 || { tail -20 gpurun_out/r6b/f32_$i.log; exit 1; }
  echo "fp32 $i $(grep metric gpurun_out/r6b/f32_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 10 > gpurun_out/r6b/bf16.log 2>&1 || { tail -20 gpurun_out/r6b/bf16.log; exit 1; }
grep metric gpurun_out/r6b/bf16.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bf16", d["ms_per_step"], d["value"], "fp32", d["fp32"])'
