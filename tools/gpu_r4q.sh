#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_native_kernels.py tests/test_conv_x8.py tests/test_resnet_block_parity.py > gpurun_out/r4q/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r4q/tests.log | tail -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/stats_ab.py > gpurun_out/r4q/stats_ab.log 2>&1 || { tail -20 gpurun_out/r4q/stats_ab.log; exit 1; }
grep '^{' gpurun_out/r4q/stats_ab.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4q/bench$i.log 2>&1 || { tail -30 gpurun_out/r4q/bench$i.log; exit 1; }
tail -1 gpurun_out/r4q/bench$i.log | cut -c1-200
done
