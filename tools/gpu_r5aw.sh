#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5aw
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5aw/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r5aw/gpu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5aw/gpu_tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aw/smoke.log 2>&1 || { tail -30 gpurun_out/r5aw/smoke.log; exit 1; }
tail -1 gpurun_out/r5aw/smoke.log
