#!/bin/bash
# u8 (offset) activations: kernel numerics test, kernel probe, then the int8 VGG16 bench, unsigned
# on / off and the calibration rule under unsigned codes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_int8_static.py -m gpu > gpurun_out/r5w/test.log 2>&1 || { tail -40 gpurun_out/r5w/test.log; exit 1; }
tail -1 gpurun_out/r5w/test.log
timeout -k 10 300 python tools/i8_power_probe.py 2>&1 | tail -6
for cfg in "1 p99.99" "0 p99.99" "1 p99.999" "1 max" "0 p99.99" "1 p99.999"; do
  set -- $cfg
  L=gpurun_out/r5w/int8_u$1_$2.log
  BIGDL_INT8_UNSIGNEDACTIVATIONS=$1 BIGDL_INT8_CALIBRATION=$2 timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 --calib 64 > $L 2>&1 || { tail -30 $L; exit 1; }
  echo "u8=$1 $2 $(grep metric $L | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["int8_over_bf16"], d["cosine_int8_vs_fp32"], d["cosine_image_dependent"], d["top1_agreement"])')"
done
