#!/bin/bash
# final numbers after the shortcut-BN deferral: bf16 x3 and the fp32 record
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ax
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_block_parity.py tests/test_fp32*.py > gpurun_out/r5ax/t.log 2>&1 || { tail -30 gpurun_out/r5ax/t.log; exit 1; }
tail -1 gpurun_out/r5ax/t.log
for i in 1 2 3; do
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 --fp32-steps 10 > gpurun_out/r5ax/b$i.log 2>&1 || { tail -20 gpurun_out/r5ax/b$i.log; exit 1; }
  echo "run $i $(grep metric gpurun_out/r5ax/b$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["fp32"]["ms_per_step"], d["fp32"]["value"])')"
done
