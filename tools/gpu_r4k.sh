#!/bin/bash
# Round 4 (k): PTB kernel profile, step kernels vs the 4-wave granule kernels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
for v in 0 7; do
  BIGDL_RNN_PERSIST=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ptb$v -o run -- python tools/bench_configs.py --config ptb --steps 10 --warmup 3 > gpurun_out/r4k/ptb_p$v.log 2>&1 || { tail -20 gpurun_out/r4k/ptb_p$v.log; exit 1; }
  db=$(find /tmp/ptb$v -name '*.db' | head -1)
  ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/r4k/ptb_p$v.log') if l.startswith('{\"metric')][-1]['ms_per_step']*10)")
  LAST_MS=$ms python tools/rocpd_summary.py "$db" 10 25 > gpurun_out/r4k/ptb_p${v}_kernels.txt
  head -16 gpurun_out/r4k/ptb_p${v}_kernels.txt | cut -c1-150
done
