#!/bin/bash
# Round 4 (n): pointwise wgrad fast gather — correctness, per-shape table, step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_native_kernels.py -k "conv" tests/test_conv_x8.py > gpurun_out/r4n/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r4n/tests.log | tail -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4n/bench.log 2>&1 || { tail -30 gpurun_out/r4n/bench.log; exit 1; }
tail -1 gpurun_out/r4n/bench.log | cut -c1-200
timeout -k 10 300 python -u tools/pw_bench.py > gpurun_out/r4n/pw.jsonl 2>&1 || { tail -20 gpurun_out/r4n/pw.jsonl; exit 1; }
tail -1 gpurun_out/r4n/pw.jsonl
