#!/bin/bash
# full GPU suite + smoke + default bench (the driver's round-end sequence)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ar
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5ar/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r5ar/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5ar/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ar/smoke.log 2>&1 || { tail -30 gpurun_out/r5ar/smoke.log; exit 1; }
tail -1 gpurun_out/r5ar/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5ar/bench_default.log 2>&1 || { tail -30 gpurun_out/r5ar/bench_default.log; exit 1; }
grep metric gpurun_out/r5ar/bench_default.log | cut -c1-400
