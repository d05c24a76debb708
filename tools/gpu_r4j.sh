#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4j
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_conv_i8_native.py -k vgg16 > gpurun_out/r4j/tests_i8.log 2>&1; rc=$?
grep -E "^E |passed|failed" gpurun_out/r4j/tests_i8.log | head -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace -d /tmp/lagdb -o run -- python bench.py --steps 3 --warmup 3 --phase-steps 0 --fp32-steps 0 > gpurun_out/r4j/lag.log 2>&1 || { tail -20 gpurun_out/r4j/lag.log; exit 1; }
db=$(find /tmp/lagdb -name '*.db' | head -1)
ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/r4j/lag.log') if l.startswith('{\"metric')][-1]['ms_per_step'])")
python tools/launch_lag.py "$db" $ms 2 > gpurun_out/r4j/lag_summary.txt 2>&1
head -50 gpurun_out/r4j/lag_summary.txt
bash tools/gpu_r4k.sh || exit 1
mkdir -p gpurun_out/r4j
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --force-distri --syncbn > gpurun_out/r4j/bench_syncbn.log 2>&1 || { tail -30 gpurun_out/r4j/bench_syncbn.log; exit 1; }
tail -1 gpurun_out/r4j/bench_syncbn.log | cut -c1-220
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4j/bench_local.log 2>&1 || { tail -30 gpurun_out/r4j/bench_local.log; exit 1; }
tail -1 gpurun_out/r4j/bench_local.log | cut -c1-220
BIGDL_WGRAD_FIRST=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4j/bench_wgfirst.log 2>&1 || { tail -30 gpurun_out/r4j/bench_wgfirst.log; exit 1; }
echo wgrad-first; tail -1 gpurun_out/r4j/bench_wgfirst.log | cut -c1-220
