#!/bin/bash
# bf16 ResNet-50 step: HBM bytes per kernel (fp32 phase off) and kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5z
timeout -k 10 600 bash tools/pmc_step_bytes.sh > gpurun_out/r5z/step_bytes.log 2>&1 || { tail -20 gpurun_out/r5z/step_bytes.log; exit 1; }
cp gpurun_out/pmcstep/summary.txt gpurun_out/r5z/step_bytes_summary.txt; rm -rf gpurun_out/pmcstep
head -3 gpurun_out/r5z/step_bytes_summary.txt
timeout -k 10 700 bash tools/prof_resnet.sh > gpurun_out/r5z/prof.log 2>&1 || { tail -20 gpurun_out/r5z/prof.log; exit 1; }
cp gpurun_out/prof_rn_summary.txt gpurun_out/r5z/
head -45 gpurun_out/r5z/prof_rn_summary.txt
