#!/bin/bash
# bf16 evidence refresh: per-shape conv table vs hipBLASLt (1x1 GEMM) and MIOpen (conv2d),
# per-kernel HBM bytes of one training step, PMC tables for the 56^2 pointwise and a 3x3 shape
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5y
MIOPEN_FIND_MODE=FAST VENDOR_CONV=1 timeout -k 10 420 python tools/pw_bench.py > gpurun_out/r5y/pw_bench.jsonl 2> gpurun_out/r5y/pw_bench.err || { tail -20 gpurun_out/r5y/pw_bench.err; exit 1; }
tail -1 gpurun_out/r5y/pw_bench.jsonl
timeout -k 10 600 bash tools/pmc_step_bytes.sh > gpurun_out/r5y/step_bytes.log 2>&1 || { tail -20 gpurun_out/r5y/step_bytes.log; exit 1; }
cp gpurun_out/pmcstep/summary.txt gpurun_out/r5y/step_bytes_summary.txt; rm -rf gpurun_out/pmcstep
head -3 gpurun_out/r5y/step_bytes_summary.txt
SPECS="64,256,1,1,56 fwdstats;64,64,1,1,56 fwdstats;128,128,3,1,28 fwdstats;64,256,1,1,56 dgrad" timeout -k 10 600 bash tools/pmc_conv2.sh > gpurun_out/r5y/pmc.log 2>&1 || { tail -20 gpurun_out/r5y/pmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/r5y/pmc_summary.txt; rm -rf gpurun_out/pmc2
head -30 gpurun_out/r5y/pmc_summary.txt
