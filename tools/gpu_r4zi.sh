#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zi
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_fp32x3.py tests/test_conv_x8.py tests/test_native_kernels.py > gpurun_out/r4zi/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r4zi/tests.log | tail -5; [ $rc -eq 0 ] || exit 1
bash tools/prof_fp32.sh > gpurun_out/r4zi/prof.log 2>&1 || { tail -20 gpurun_out/r4zi/prof.log; exit 1; }
cp gpurun_out/prof_f32_summary.txt gpurun_out/r4zi/
head -30 gpurun_out/r4zi/prof_f32_summary.txt | cut -c1-160
tail -1 gpurun_out/prof_f32.log | cut -c1-200
