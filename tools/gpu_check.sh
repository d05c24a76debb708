#!/bin/bash
# One GPU round: native-kernel tests, bench, optional conv microbench and rocprofv3 kernel stats.
# Each GPU step has its own timeout; steps are chained so a failure stops the script.
# Env knobs (set inside the gpurun command): STEPS, PROFILE=0|1, CONVBENCH=0|1, TESTS=0|1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then echo "pytest gpu failed rc=$rc"; exit $rc; fi
fi
if [ "${CONVBENCH:-0}" = "1" ]; then
  timeout -k 10 300 python tools/bench_conv.py --no-miopen > gpurun_out/bench_conv.log 2>&1 || { tail -20 gpurun_out/bench_conv.log; exit 1; }
  tail -1 gpurun_out/bench_conv.log
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
  echo profiled
fi
