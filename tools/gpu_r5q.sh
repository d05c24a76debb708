#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5q
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_int8_static.py tests/test_quantized.py tests/test_syncbn_native.py tests/test_rnn_fp32.py tests/test_lstm_stack.py > gpurun_out/r5q/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r5q/tests.log | tail -8; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r5q/int8.log 2>&1 || { tail -30 gpurun_out/r5q/int8.log; exit 1; }
grep metric gpurun_out/r5q/int8.log | cut -c1-900
for rep in 1 2 3; do
for cfg in local syncbn syncmr; do
  export BIGDL_BN_SYNCONERANKLOCAL=1
  case $cfg in local) a="";; syncbn) a="--force-distri --syncbn";; syncmr) a="--force-distri --syncbn"; export BIGDL_BN_SYNCONERANKLOCAL=0;; esac
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 $a > gpurun_out/r5q/bench_${cfg}_$rep.log 2>&1 || { tail -30 gpurun_out/r5q/bench_${cfg}_$rep.log; exit 1; }
  echo "$cfg $rep $(tail -1 gpurun_out/r5q/bench_${cfg}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
done
bash tools/prof_infer.sh
bash tools/prof_step_dispatch.sh
