#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_syncbn_native.py tests/test_resnet_block_parity.py > gpurun_out/r4p/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r4p/tests.log | tail -5; [ $rc -eq 0 ] || exit 1
for cfg in local syncbn distri; do
  case $cfg in local) a="";; syncbn) a="--force-distri --syncbn";; distri) a="--force-distri --comm-dtype bf16";; esac
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 $a > gpurun_out/r4p/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/r4p/bench_$cfg.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r4p/bench_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
