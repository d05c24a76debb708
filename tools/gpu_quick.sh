#!/bin/bash
# GPU tests + 1-GPU bench + kernel-stat profile + roctx marker trace; PMC on two conv shapes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
PROFILE=0 bash tools/gpu_check.sh && bash tools/prof_resnet.sh || exit 1
timeout -k 10 300 env BIGDL_ROCTX=1 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/r2/prof_mark -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/r2/prof_mark.log 2>&1 || { tail -20 gpurun_out/r2/prof_mark.log; exit 1; }
python tools/marker_summary.py gpurun_out/r2/prof_mark 5 > gpurun_out/r2/marker_summary.txt; head -12 gpurun_out/r2/marker_summary.txt
rm -f gpurun_out/r2/prof_mark/*kernel_trace.csv
if [ "${PMC:-1}" = "1" ]; then
  rm -rf gpurun_out/pmc2; SPECS='256,1024,1,1,14 fwdstats;64,256,1,1,56 fwdstats' bash tools/pmc_conv2.sh && python tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/pmc2_summary.txt || exit 1
fi
