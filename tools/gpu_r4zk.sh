#!/bin/bash
# Round 4 (z): full GPU suite (no -x), smoke(), then the driver's default bench (bf16 headline + fp32 record).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zk
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4zk/tests_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r4zk/tests_gpu.log | tail -15; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4zk/smoke.log 2>&1 || { tail -20 gpurun_out/r4zk/smoke.log; exit 1; }
tail -1 gpurun_out/r4zk/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4zk/bench.log 2>&1 || { tail -30 gpurun_out/r4zk/bench.log; exit 1; }
tail -1 gpurun_out/r4zk/bench.log
