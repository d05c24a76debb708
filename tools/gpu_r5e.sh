#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool32.py tests/test_fp32_direct.py > gpurun_out/r5e/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r5e/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5d.sh
