#!/bin/bash
# ResNet-50 bf16 training step: per-dispatch listing (name, grid, duration) of the last step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_sd -o run -- python3 bench.py --steps 3 --warmup 3 --fp32-steps 0 --phase-steps 0 $BARGS > gpurun_out/prof_sd.log 2>&1 || { tail -20 gpurun_out/prof_sd.log; exit 1; }
db=$(find gpurun_out/prof_sd -name '*.db' | head -1)
python3 tools/rocpd_dispatches.py "$db" ${NDISP:-500} > gpurun_out/prof_step_dispatches.txt; rm -rf gpurun_out/prof_sd
grep metric gpurun_out/prof_sd.log | cut -c1-200
wc -l gpurun_out/prof_step_dispatches.txt
