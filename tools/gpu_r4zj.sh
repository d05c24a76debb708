#!/bin/bash
# fp32 A/B: conv-epilogue BN statistics on / off (bigdl.fp32.convStats), bench fp32 timing, twice each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zj
for i in 1 2; do
for v in 1 0; do
BIGDL_FP32_CONVSTATS=$v timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --phase-steps 0 --fp32-steps 0 > gpurun_out/r4zj/b_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r4zj/b_${v}_$i.log; exit 1; }
echo "convStats=$v $(tail -1 gpurun_out/r4zj/b_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
done
