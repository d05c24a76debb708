#!/bin/bash
# ResNet-50 fp32 step (bf16x3 native path): rocprofv3 kernel stats normalised to one step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
BIGDL_FP32_NATIVE=${NATIVE:-1} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python bench.py --dtype fp32 --steps 3 --warmup 2 --phase-steps 0 --fp32-steps 0 > gpurun_out/prof_f32.log 2>&1 || { tail -20 gpurun_out/prof_f32.log; exit 1; }
db=$(find gpurun_out/prof_f32 -name '*.db' | head -1)
ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/prof_f32.log') if l.startswith('{\"metric')][-1]['ms_per_step']*3)")
LAST_MS=$ms python tools/rocpd_summary.py "$db" 3 ${TOP:-40} > gpurun_out/prof_f32_summary.txt; rm -rf gpurun_out/prof_f32
head -${TOP:-50} gpurun_out/prof_f32_summary.txt; grep -c "at::native" gpurun_out/prof_f32_summary.txt || true
