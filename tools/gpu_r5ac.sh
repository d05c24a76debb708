#!/bin/bash
# bench.py bf16 repeats (same box)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ac
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5ac/b$i.log 2>&1 || { tail -20 gpurun_out/r5ac/b$i.log; exit 1; }
  echo "bf16 $i $(grep metric gpurun_out/r5ac/b$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
