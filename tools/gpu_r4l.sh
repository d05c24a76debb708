#!/bin/bash
# Round 4 (l): full GPU suite with the new defaults, bench, step profile + timeline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4l
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4l/tests_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r4l/tests_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r4l/bench.log 2>&1 || { tail -30 gpurun_out/r4l/bench.log; exit 1; }
tail -1 gpurun_out/r4l/bench.log
bash tools/prof_resnet.sh || exit 1
cp gpurun_out/prof_rn_summary.txt gpurun_out/r4l/
bash tools/prof_timeline.sh r4l --fp32-steps 0 || exit 1
cp gpurun_out/prof_r4l_summary.txt gpurun_out/prof_r4l_timeline.txt gpurun_out/r4l/ && rm -f gpurun_out/prof_r4l.db
