#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_resnet_block_parity.py tests/test_native_kernels.py tests/test_bn_prologue.py tests/test_no_fallback.py tests/test_syncbn_native.py tests/test_fp32_direct.py tests/test_compiled.py > gpurun_out/r5t/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r5t/tests.log | tail -8; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for f in 1 0; do
  BIGDL_BN_FOLDFINALIZE=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5t/bench_${f}_$rep.log 2>&1 || { tail -30 gpurun_out/r5t/bench_${f}_$rep.log; exit 1; }
  echo "fold=$f $rep $(tail -1 gpurun_out/r5t/bench_${f}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))')"
done
done
