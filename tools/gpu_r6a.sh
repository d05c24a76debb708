#!/bin/bash
# round 6: fp32 step with the side-stream fp32 wgrad + unrolled fp32 BN apply; fp32 tests; profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_direct.py tests/test_fp32x3.py tests/test_pool32.py tests/test_rnn_fp32.py tests/test_no_fallback.py tests/test_native_kernels.py > gpurun_out/r6a/tests.log 2>&1 || { tail -30 gpurun_out/r6a/tests.log; exit 1; }
tail -3 gpurun_out/r6a/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > gpurun_out/r6a/f32_$i.log 2>&1 || { tail -20 gpurun_out/r6a/f32_$i.log; exit 1; }
  echo "fp32 $i $(grep metric gpurun_out/r6a/f32_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
done
bash tools/prof_fp32.sh > /dev/null && cp gpurun_out/prof_f32_summary.txt gpurun_out/r6a/ && head -45 gpurun_out/r6a/prof_f32_summary.txt
