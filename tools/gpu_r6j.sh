#!/bin/bash
# fp32 parity (well-conditioned), full GPU suite (no -x), bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -s -v --timeout 300 --timeout-method thread tests/test_train_parity.py -k fp32 > $O/parity.log 2>&1; rc=$?
grep -A3 "fp32 ResNet-50" $O/parity.log; tail -3 $O/parity.log
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1
bash tools/prof_fp32.sh > /dev/null && cp gpurun_out/prof_f32_summary.txt $O/ && head -60 $O/prof_f32_summary.txt
