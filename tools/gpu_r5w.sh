#!/bin/bash
# u8 (offset) activations: kernel numerics test, then the int8 VGG16 bench with unsigned on / off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_int8_static.py -m gpu > gpurun_out/r5w/test.log 2>&1 || { tail -40 gpurun_out/r5w/test.log; exit 1; }
tail -3 gpurun_out/r5w/test.log
for u in 1 0 1; do
  BIGDL_INT8_UNSIGNEDACTIVATIONS=$u timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 --calib 64 > gpurun_out/r5w/int8_u$u.log 2>&1 || { tail -30 gpurun_out/r5w/int8_u$u.log; exit 1; }
  echo "u8=$u $(grep metric gpurun_out/r5w/int8_u$u.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["int8_over_bf16"], d["cosine_int8_vs_fp32"], d["cosine_image_dependent"], d["top1_agreement"])')"
done
