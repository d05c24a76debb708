#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6bd
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v -s -m gpu --timeout 400 --timeout-method thread tests/test_distri_gpu_rehearsal.py > $O/tests.log 2>&1; rc=$?
grep -v INFO $O/tests.log | grep -i "rel=\|passed\|failed\|error\|assert" | head -30
exit $rc
