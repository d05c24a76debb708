#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
for cal in max p99.999 p99.99 p99.9; do
  BIGDL_INT8_CALIBRATION=$cal timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r5u/int8_$cal.log 2>&1 || { tail -30 gpurun_out/r5u/int8_$cal.log; exit 1; }
  echo "$cal $(grep metric gpurun_out/r5u/int8_$cal.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["int8_over_bf16"], d["cosine_int8_vs_fp32"], d["cosine_image_dependent"], d["top1_agreement"])')"
done
