#!/bin/bash
# full GPU suite, bench repeats and the step kernel summary after the store-pass / int8 changes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5aj
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5aj/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r5aj/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5aj/gpu_tests.log
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5aj/b$i.log 2>&1 || { tail -20 gpurun_out/r5aj/b$i.log; exit 1; }
  echo "bf16 $i $(grep metric gpurun_out/r5aj/b$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 700 bash tools/prof_resnet.sh > gpurun_out/r5aj/prof.log 2>&1 || { tail -20 gpurun_out/r5aj/prof.log; exit 1; }
cp gpurun_out/prof_rn_summary.txt gpurun_out/r5aj/
head -30 gpurun_out/r5aj/prof_rn_summary.txt
