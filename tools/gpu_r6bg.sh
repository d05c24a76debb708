#!/bin/bash
# fp32 ResNet-50 step after the torch-kernel removal, 3 repeats on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6bg
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > $O/f32_$i.log 2>&1 || { tail -30 $O/f32_$i.log; exit 1; }
  tail -1 $O/f32_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fp32", d["ms_per_step"], d["value"])'
done
