#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ay
for i in 1 2 3; do
  for v in 1 0; do
    BIGDL_WGRAD_EXTRA=$v timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5ay/b${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5ay/b${v}_$i.log; exit 1; }
    echo "wgextra=$v $i $(grep metric gpurun_out/r5ay/b${v}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
