#!/bin/bash
# Compile-phase kernel selection: GPU tests of nn/compiled.py, then ResNet-50 inference eager vs
# tuned eager vs compiled (tuned + HIP graph).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_compiled.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3e/pytest.log 2>&1 || { tail -40 gpurun_out/r3e/pytest.log; exit 1; }
tail -1 gpurun_out/r3e/pytest.log
timeout -k 10 500 python tools/bench_infer.py > gpurun_out/r3e/infer.jsonl 2> gpurun_out/r3e/infer.err || { tail -20 gpurun_out/r3e/infer.err; exit 1; }
cat gpurun_out/r3e/infer.jsonl
