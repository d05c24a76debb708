#!/bin/bash
# Round 4 (c): BN one-launch finalize+apply (atomic statistics) parity, attention / int8 kernels,
# then the bench (bf16 headline + fp32 record), the step profile and the int8 VGG16 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_resnet_block_parity.py tests/test_native_kernels.py tests/test_bn_prologue.py tests/test_syncbn_native.py > gpurun_out/r4c/tests_bn.log 2>&1 || { tail -40 gpurun_out/r4c/tests_bn.log; exit 1; }
tail -2 gpurun_out/r4c/tests_bn.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4c/bench.log 2>&1 || { tail -30 gpurun_out/r4c/bench.log; exit 1; }
tail -1 gpurun_out/r4c/bench.log
timeout -k 10 300 $T tests/test_attn_decode_native.py tests/test_attention_native.py tests/test_attention_module_native.py > gpurun_out/r4c/tests_attn.log 2>&1 || { tail -40 gpurun_out/r4c/tests_attn.log; exit 1; }
tail -2 gpurun_out/r4c/tests_attn.log
timeout -k 10 300 $T tests/test_conv_i8_native.py tests/test_quantized.py > gpurun_out/r4c/tests_i8.log 2>&1 || { tail -40 gpurun_out/r4c/tests_i8.log; exit 1; }
tail -2 gpurun_out/r4c/tests_i8.log
timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r4c/int8.log 2>&1 || { tail -30 gpurun_out/r4c/int8.log; exit 1; }
tail -1 gpurun_out/r4c/int8.log
bash tools/prof_resnet.sh || exit 1
cp gpurun_out/prof_rn_summary.txt gpurun_out/r4c/
