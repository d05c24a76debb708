#!/bin/bash
# Compiled ResNet-50 inference (BS, default 256): rocprofv3 kernel stats of the steady-state window.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inf -o run -- python3 tools/infer_one.py > gpurun_out/prof_inf.log 2>&1 || { tail -20 gpurun_out/prof_inf.log; exit 1; }
db=$(find gpurun_out/prof_inf -name '*.db' | head -1)
ms=$(python3 -c "import json; print([json.loads(l) for l in open('gpurun_out/prof_inf.log') if l.startswith('{\"batch')][-1]['ms']*20)")
LAST_MS=$ms python3 tools/rocpd_summary.py "$db" 20 40 > gpurun_out/prof_inf_summary.txt
python3 tools/rocpd_dispatches.py "$db" ${NDISP:-70} > gpurun_out/prof_inf_dispatches.txt; rm -rf gpurun_out/prof_inf
grep batch gpurun_out/prof_inf.log
head -50 gpurun_out/prof_inf_summary.txt
