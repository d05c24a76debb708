#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool32.py tests/test_fp32_direct.py tests/test_fp32x3.py > gpurun_out/r5f/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r5f/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 --phase-steps 0 > gpurun_out/r5f/bench_f32.log 2>&1 || { tail -20 gpurun_out/r5f/bench_f32.log; exit 1; }
tail -1 gpurun_out/r5f/bench_f32.log | cut -c1-300
bash tools/prof_fp32.sh > /dev/null && cp gpurun_out/prof_f32_summary.txt gpurun_out/r5f/ && head -42 gpurun_out/r5f/prof_f32_summary.txt
