#!/bin/bash
# split-K GEMM: numerics, then int8 VGG16 (bf16 FC head) and the GEMM-using tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ap
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gemm_rnn.py tests/test_conv_i8_native.py > gpurun_out/r5ap/test.log 2>&1 || { tail -40 gpurun_out/r5ap/test.log; exit 1; }
tail -1 gpurun_out/r5ap/test.log
for i in 1 2; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 --calib 64 > gpurun_out/r5ap/int8_$i.log 2>&1 || { tail -30 gpurun_out/r5ap/int8_$i.log; exit 1; }
  echo "int8 $i $(grep metric gpurun_out/r5ap/int8_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["int8_over_bf16"], d["bf16"], d["fp32"], d["cosine_int8_vs_fp32"])')"
done
