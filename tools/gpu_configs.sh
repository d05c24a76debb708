#!/bin/bash
# Secondary-config benches (tools/bench_configs.py) + per-config rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CONFIGS:-lenet vgg ptb inception}; do
  timeout -k 10 300 python tools/bench_configs.py --config $c > gpurun_out/cfg_$c.log 2>&1 || { tail -30 gpurun_out/cfg_$c.log; exit 1; }
  tail -1 gpurun_out/cfg_$c.log
done
if [ "${PROFILE:-1}" = "1" ]; then
  for c in ${PCONFIGS:-vgg ptb inception}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run -- python tools/bench_configs.py --config $c --steps 5 --warmup 2 > gpurun_out/prof_$c.log 2>&1 || { tail -20 gpurun_out/prof_$c.log; exit 1; }
    db=$(find gpurun_out/prof_$c -name '*.db' | head -1)
    ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/prof_$c.log') if l.startswith('{\"metric')][-1]['ms_per_step']*5)")
    LAST_MS=$ms python tools/rocpd_summary.py "$db" 5 30 > gpurun_out/prof_${c}_summary.txt; rm -rf gpurun_out/prof_$c
    head -8 gpurun_out/prof_${c}_summary.txt
  done
fi
