#!/bin/bash
# Round 4 (o): kernel profiles of the world-1 SyncBN and bf16-wire DistriOptimizer steps vs local.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4o
for cfg in local syncbn distri; do
  case $cfg in local) a="";; syncbn) a="--force-distri --syncbn";; distri) a="--force-distri --comm-dtype bf16";; esac
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/p_$cfg -o run -- python bench.py --steps 5 --warmup 3 --fp32-steps 0 --phase-steps 0 $a > gpurun_out/r4o/$cfg.log 2>&1 || { tail -20 gpurun_out/r4o/$cfg.log; exit 1; }
  db=$(find /tmp/p_$cfg -name '*.db' | head -1)
  ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/r4o/$cfg.log') if l.startswith('{\"metric')][-1]['ms_per_step']*5)")
  LAST_MS=$ms python tools/rocpd_summary.py "$db" 5 60 > gpurun_out/r4o/${cfg}_kernels.txt
  echo "$cfg $(head -1 gpurun_out/r4o/${cfg}_kernels.txt) $(tail -1 gpurun_out/r4o/$cfg.log | cut -c150-230)"
done
