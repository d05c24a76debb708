#!/bin/bash
# round 6 re-entry: full GPU suite + default bench (bf16 headline + fp32 record) + fp32 kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1
bash tools/prof_fp32.sh > /dev/null && cp gpurun_out/prof_f32_summary.txt $O/ && head -60 $O/prof_f32_summary.txt
