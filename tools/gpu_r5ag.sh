#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ag
SPECS="64,64,3,1,56 fwd" timeout -k 10 300 bash tools/pmc_conv2.sh > gpurun_out/r5ag/pmc.log 2>&1 || { tail -20 gpurun_out/r5ag/pmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/r5ag/pmc_summary.txt; rm -rf gpurun_out/pmc2
cat gpurun_out/r5ag/pmc_summary.txt
