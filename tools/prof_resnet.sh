#!/bin/bash
# ResNet-50 training step: bench + rocprofv3 kernel stats normalised to one step (summary only).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run -- python bench.py --steps 5 --warmup 3 --fp32-steps 0 --phase-steps 0 $BARGS > gpurun_out/prof_rn.log 2>&1 || { tail -20 gpurun_out/prof_rn.log; exit 1; }
db=$(find gpurun_out/prof_rn -name '*.db' | head -1)
ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/prof_rn.log') if l.startswith('{\"metric')][-1]['ms_per_step']*5)")
LAST_MS=$ms python tools/rocpd_summary.py "$db" 5 40 > gpurun_out/prof_rn_summary.txt; rm -rf gpurun_out/prof_rn
head -60 gpurun_out/prof_rn_summary.txt
