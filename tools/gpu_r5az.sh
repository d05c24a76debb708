#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5az
for i in 1 2 3; do
  for v in 1024 2048 512; do
    BIGDL_BN_APPLY_BLOCKS=$v timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5az/b${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5az/b${v}_$i.log; exit 1; }
    echo "applyblocks=$v $i $(grep metric gpurun_out/r5az/b${v}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
