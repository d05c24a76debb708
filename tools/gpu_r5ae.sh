#!/bin/bash
# halo-patch 64->64 3x3 kernel: numerics, then timing (on / off) and the bf16 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ae
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_patch.py > gpurun_out/r5ae/test.log 2>&1 || { tail -40 gpurun_out/r5ae/test.log; exit 1; }
tail -2 gpurun_out/r5ae/test.log
for v in 1 0; do
  BIGDL_CONV_PATCH=$v ONLY3=1 timeout -k 10 300 python tools/pw_bench.py > gpurun_out/r5ae/pw3_patch$v.jsonl 2>&1 || { tail -20 gpurun_out/r5ae/pw3_patch$v.jsonl; exit 1; }
  head -1 gpurun_out/r5ae/pw3_patch$v.jsonl | cut -c1-200
done
