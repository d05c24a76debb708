#!/bin/bash
# 256x256 x8 tile: numerics, then per-shape timings with BIGDL_CONV_X8=2 vs 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_x8.py > gpurun_out/r5ab/test.log 2>&1 || { tail -40 gpurun_out/r5ab/test.log; exit 1; }
tail -2 gpurun_out/r5ab/test.log
for v in 2 1; do
  BIGDL_CONV_X8=$v timeout -k 10 400 python tools/pw_bench.py > gpurun_out/r5ab/pw_x8_$v.jsonl 2>&1 || { tail -20 gpurun_out/r5ab/pw_x8_$v.jsonl; exit 1; }
  tail -1 gpurun_out/r5ab/pw_x8_$v.jsonl
done
