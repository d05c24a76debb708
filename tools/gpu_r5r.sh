#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5r
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_resnet_block_parity.py tests/test_native_kernels.py tests/test_bn_prologue.py tests/test_conv_x8.py tests/test_no_fallback.py tests/test_stem_input.py > gpurun_out/r5r/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r5r/tests.log | tail -8; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5r/bench_$rep.log 2>&1 || { tail -30 gpurun_out/r5r/bench_$rep.log; exit 1; }
  echo "bf16 $rep $(tail -1 gpurun_out/r5r/bench_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
bash tools/prof_step_dispatch.sh
