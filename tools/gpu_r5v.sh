#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v
for cfg in "p99.99 1" "p99.99 0" "p99.999 0" "max 0"; do
  set -- $cfg
  BIGDL_INT8_CALIBRATION=$1 BIGDL_INT8_QUANTIZELINEAR=$2 timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 --calib 64 > gpurun_out/r5v/int8_$1_$2.log 2>&1 || { tail -30 gpurun_out/r5v/int8_$1_$2.log; exit 1; }
  echo "$1 lin=$2 $(grep metric gpurun_out/r5v/int8_$1_$2.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["int8_over_bf16"], d["cosine_int8_vs_fp32"], d["cosine_image_dependent"], d["top1_agreement"])')"
done
