#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4s
bash tools/prof_fp32.sh > gpurun_out/r4s/prof.log 2>&1 || { tail -20 gpurun_out/r4s/prof.log; exit 1; }
cp gpurun_out/prof_f32_summary.txt gpurun_out/r4s/
head -45 gpurun_out/r4s/prof_f32_summary.txt | cut -c1-160
tail -1 gpurun_out/prof_f32.log | cut -c1-200
