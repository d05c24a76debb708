#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp32_direct.py tests/test_compiled.py tests/test_pool32.py > gpurun_out/r5i/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5i/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_x3.py --out gpurun_out/r5i/bench_x3.jsonl 2>&1 | grep -v amdgpu.ids > gpurun_out/r5i/bench_x3.log; tail -2 gpurun_out/r5i/bench_x3.log
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 --phase-steps 0 > gpurun_out/r5i/bench_f32.log 2>&1 || { tail -20 gpurun_out/r5i/bench_f32.log; exit 1; }
tail -1 gpurun_out/r5i/bench_f32.log | cut -c1-250
timeout -k 10 400 python -u tools/bench_infer.py > gpurun_out/r5i/infer.log 2>&1; cat gpurun_out/r5i/infer.log | grep batch
