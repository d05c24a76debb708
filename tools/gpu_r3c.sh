#!/bin/bash
# fp32 compute mode (bf16x3 on the MFMA kernels): GPU tests, then ResNet-50 fp32 step native vs torch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u -m pytest tests/test_fp32x3.py tests/test_conv3d_native.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3c/pytest.log 2>&1 || { tail -40 gpurun_out/r3c/pytest.log; exit 1; }
tail -2 gpurun_out/r3c/pytest.log
for mode in 1 0; do
  BIGDL_FP32_NATIVE=$mode timeout -k 10 400 python bench.py --dtype fp32 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/r3c/bench_fp32_native$mode.log 2>&1 || { tail -30 gpurun_out/r3c/bench_fp32_native$mode.log; exit 1; }
  echo "fp32 native=$mode: $(tail -1 gpurun_out/r3c/bench_fp32_native$mode.log)"
done
