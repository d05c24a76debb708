#!/bin/bash
# VGG16 int8 / bf16 / fp32 inference (tools/bench_configs.py --config int8): rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_i8 -o run -- python3 tools/bench_configs.py --config int8 --steps 5 --warmup 2 > gpurun_out/prof_i8.log 2>&1 || { tail -20 gpurun_out/prof_i8.log; exit 1; }
db=$(find gpurun_out/prof_i8 -name '*.db' | head -1)
python3 tools/rocpd_summary.py "$db" 1 45 > gpurun_out/prof_i8_summary.txt
python3 tools/rocpd_dispatches.py "$db" ${NDISP:-60} > gpurun_out/prof_i8_dispatches.txt; rm -rf gpurun_out/prof_i8
grep metric gpurun_out/prof_i8.log | cut -c1-600
head -50 gpurun_out/prof_i8_summary.txt
