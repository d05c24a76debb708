#!/bin/bash
# x8 (256x128 LDS-DMA 32x32x16) kernel on the 3x3 shapes: timings and PMC counters
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5aa
BIGDL_CONV_X8=1 ONLY3=1 timeout -k 10 300 python tools/pw_bench.py > gpurun_out/r5aa/pw3_x8.jsonl 2>&1 || { tail -20 gpurun_out/r5aa/pw3_x8.jsonl; exit 1; }
cut -c1-220 gpurun_out/r5aa/pw3_x8.jsonl
export BIGDL_CONV_X8=1
SPECS="256,256,3,1,14 fwd;64,64,3,1,56 fwd;512,512,3,1,7 fwd" timeout -k 10 600 bash tools/pmc_conv2.sh > gpurun_out/r5aa/pmc.log 2>&1 || { tail -20 gpurun_out/r5aa/pmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/r5aa/pmc_summary.txt; rm -rf gpurun_out/pmc2
cat gpurun_out/r5aa/pmc_summary.txt
