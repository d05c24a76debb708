#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4r
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_compiled.py > gpurun_out/r4r/tests.log 2>&1; rc=$?
grep -E "^E  |FAILED|passed|failed" gpurun_out/r4r/tests.log | tail -8; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python tools/bench_infer.py > gpurun_out/r4r/infer.log 2>&1 || { tail -20 gpurun_out/r4r/infer.log; exit 1; }
tail -6 gpurun_out/r4r/infer.log
