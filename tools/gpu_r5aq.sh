#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5aq
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_int8_static.py tests/test_conv_i8_native.py tests/test_native_kernels.py -k "int8 or i8 or stem or conv" > gpurun_out/r5aq/test.log 2>&1 || { tail -40 gpurun_out/r5aq/test.log; exit 1; }
tail -1 gpurun_out/r5aq/test.log
for i in 1 2; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 --calib 64 > gpurun_out/r5aq/int8_$i.log 2>&1 || { tail -30 gpurun_out/r5aq/int8_$i.log; exit 1; }
  echo "int8 $i $(grep metric gpurun_out/r5aq/int8_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["int8_over_bf16"], d["bf16"], d["cosine_int8_vs_fp32"], d["top1_agreement"])')"
done
