#!/bin/bash
# Round 4: x8 (32x32x16 / LDS-DMA) conv family — numerics first, then the full GPU suite, the bench,
# and the per-shape table with the family off / on (separate processes: the switch is read once).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u -m pytest tests/test_conv_x8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a/x8_tests.log 2>&1 || { tail -40 gpurun_out/r4a/x8_tests.log; exit 1; }
tail -3 gpurun_out/r4a/x8_tests.log
PROFILE=0 bash tools/gpu_check.sh || exit 1
for v in 0 1; do
  BIGDL_CONV_X8=$v timeout -k 10 300 python -u tools/pw_bench.py > gpurun_out/r4a/pw_x8_$v.jsonl 2>&1 || { tail -20 gpurun_out/r4a/pw_x8_$v.jsonl; exit 1; }
  tail -1 gpurun_out/r4a/pw_x8_$v.jsonl
done
BIGDL_CONV_X8=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a/bench_x8.log 2>&1 || { tail -30 gpurun_out/r4a/bench_x8.log; exit 1; }
tail -1 gpurun_out/r4a/bench_x8.log
