#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5am
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_kernels.py tests/test_pool32.py -k "pool" > gpurun_out/r5am/test.log 2>&1 || { tail -40 gpurun_out/r5am/test.log; exit 1; }
tail -1 gpurun_out/r5am/test.log
NDISP=420 timeout -k 10 500 bash tools/prof_step_dispatch.sh > gpurun_out/r5am/sd.log 2>&1 || { tail -20 gpurun_out/r5am/sd.log; exit 1; }
grep -i "maxpool" gpurun_out/prof_step_dispatches.txt | cut -c1-90
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5am/b$i.log 2>&1 || { tail -20 gpurun_out/r5am/b$i.log; exit 1; }
  echo "bf16 $i $(grep metric gpurun_out/r5am/b$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
