#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5o
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_lstm_stack.py tests/test_native_gemm_rnn.py tests/test_rnn_persistent.py > gpurun_out/r5o/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r5o/tests.log | tail -8; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for cfg in stack nostack; do
  case $cfg in stack) v=1;; nostack) v=0;; esac
  BIGDL_FUSION_LSTMSTACK=$v timeout -k 10 300 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 > gpurun_out/r5o/ptb_${cfg}_$rep.log 2>&1 || { tail -30 gpurun_out/r5o/ptb_${cfg}_$rep.log; exit 1; }
  echo "$cfg $rep $(grep metric gpurun_out/r5o/ptb_${cfg}_$rep.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
done
