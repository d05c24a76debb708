#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zd
T="python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_learning.py"
timeout -k 10 200 $T -rA > gpurun_out/r4zd/a.log 2>&1; rc=$?; grep -E "passed|failed|^E " gpurun_out/r4zd/a.log | tail -4; exit $rc
