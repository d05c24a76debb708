#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4za
T="python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_learning.py"
timeout -k 10 200 $T > gpurun_out/r4za/a.log 2>&1; echo "default rc=$?"; grep -E "passed|failed|Error:|assert" gpurun_out/r4za/a.log | tail -4
BIGDL_CONV_X8_ILV=0 timeout -k 10 200 $T > gpurun_out/r4za/b.log 2>&1; echo "ilv0 rc=$?"; grep -E "passed|failed|Error:|assert" gpurun_out/r4za/b.log | tail -4
