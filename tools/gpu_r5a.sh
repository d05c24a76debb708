#!/bin/bash
# Round-5 baseline: bf16 headline + fp32 (10 steps) bench, then the fp32 step kernel profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 10 > gpurun_out/r5a/bench.log 2>&1 || { tail -20 gpurun_out/r5a/bench.log; exit 1; }
tail -1 gpurun_out/r5a/bench.log
bash tools/prof_fp32.sh && cp gpurun_out/prof_f32_summary.txt gpurun_out/r5a/
