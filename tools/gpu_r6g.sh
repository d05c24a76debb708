#!/bin/bash
# fp32 BN apply knobs in isolation
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6g
for u in 4 1 2 8; do
  for b in 0 1024 4096 8192; do
    BIGDL_BN32_UNROLL=$u BIGDL_BN32_BLOCKS=$b timeout -k 10 120 python tools/bench_bn32.py > gpurun_out/r6g/u${u}_b${b}.log 2>&1 || { tail -20 gpurun_out/r6g/u${u}_b${b}.log; exit 1; }
    tail -1 gpurun_out/r6g/u${u}_b${b}.log
  done
done
cat gpurun_out/r6g/u4_b0.log
