#!/bin/bash
# ResNet-50 step under rocprofv3 --kernel-trace: per-kernel summary + per-stream timeline of the last steps.
# Usage: tools/prof_timeline.sh TAG [bench args...]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-tl}; shift
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_$tag -o run -- python bench.py --steps 8 --warmup 4 --phase-steps 0 "$@" > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
db=$(find gpurun_out/prof_$tag -name '*.db' | head -1)
ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/prof_$tag.log') if l.startswith('{\"metric')][-1]['ms_per_step'])")
LAST_MS=$(python -c "print($ms*4)") python tools/rocpd_summary.py "$db" 4 45 > gpurun_out/prof_${tag}_summary.txt
python tools/timeline_step.py "$db" $ms 4 --list > gpurun_out/prof_${tag}_timeline.txt
cp "$db" gpurun_out/prof_${tag}.db
rm -rf gpurun_out/prof_$tag
head -8 gpurun_out/prof_${tag}_summary.txt; head -8 gpurun_out/prof_${tag}_timeline.txt
