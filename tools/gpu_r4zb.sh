#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zb
T="python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_fp32x3.py tests/test_gpu_learning.py > gpurun_out/r4zb/a.log 2>&1; echo "fp32x3+learn rc=$?"; grep -E "passed|failed|^E " gpurun_out/r4zb/a.log | tail -3
timeout -k 10 300 $T tests/test_attention.py tests/test_attention_module_native.py tests/test_attention_native.py tests/test_attn_decode_native.py tests/test_bn_prologue.py tests/test_compiled.py tests/test_conv3d_native.py tests/test_conv_i8_native.py tests/test_conv_x8.py tests/test_gpu_learning.py > gpurun_out/r4zb/b.log 2>&1; echo "early+learn rc=$?"; grep -E "passed|failed|^E " gpurun_out/r4zb/b.log | tail -3
