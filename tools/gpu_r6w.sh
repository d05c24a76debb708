#!/bin/bash
# new tests first, then the full GPU suite + smoke + default bench (round-6 checkpoint)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6w
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_fp32_direct.py tests/test_train_parity.py tests/test_fp32_bn_prologue.py tests/test_conv_i8_native.py > $O/new_tests.log 2>&1 || { grep -v INFO $O/new_tests.log | tail -40; exit 1; }
tail -1 $O/new_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-600
