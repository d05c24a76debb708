#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp32_direct.py tests/test_no_fallback.py > gpurun_out/r5j/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5j/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 --phase-steps 0 > gpurun_out/r5j/bench_f32_$i.log 2>&1 || { tail -20 gpurun_out/r5j/bench_f32_$i.log; exit 1; }
tail -1 gpurun_out/r5j/bench_f32_$i.log | cut -c1-200
done
bash tools/prof_fp32.sh
