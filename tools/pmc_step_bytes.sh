#!/bin/bash
# HBM bytes of one ResNet-50 training step, per kernel: two rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE: TCC counters, one derived metric per pass), summarised by tools/pmc_step_summary.py
# over the dispatches between the last two optimizer kernels (= exactly one step).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcstep
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmcstep/$c -o run -- python3 bench.py --steps 2 --warmup 2 --phase-steps 0 --fp32-steps 0 "$@" > gpurun_out/pmcstep/$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/pmcstep/$c.log; exit 1; }
done
python3 tools/pmc_step_summary.py gpurun_out/pmcstep > gpurun_out/pmcstep/summary.txt
find gpurun_out/pmcstep -name "*.db" -delete
head -40 gpurun_out/pmcstep/summary.txt
