#!/bin/bash
# int8 VGG16 per-dispatch profile (defaults: calibrated, unsigned activations, bf16 FC head)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ao
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ao/p -o run -- python3 tools/bench_configs.py --config int8 --steps 5 --warmup 2 --calib 64 > gpurun_out/r5ao/run.log 2>&1 || { tail -20 gpurun_out/r5ao/run.log; exit 1; }
db=$(find gpurun_out/r5ao/p -name '*.db' | head -1)
python3 tools/rocpd_dispatches.py "$db" 200 > gpurun_out/r5ao/disp.txt; rm -rf gpurun_out/r5ao/p
tail -40 gpurun_out/r5ao/disp.txt | cut -c1-110
