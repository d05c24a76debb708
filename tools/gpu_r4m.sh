#!/bin/bash
# Round 4 (m): full GPU suite (no -x) with the new defaults.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4m/tests_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r4m/tests_gpu.log | tail -15; [ $rc -le 1 ] || exit $rc
