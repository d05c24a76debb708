#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_direct.py > gpurun_out/r5h/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5h/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_x3.py --out gpurun_out/r5h/bench_x3.jsonl 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5h/bench_x3.log
