#!/bin/bash
# Round 4 (c): BN one-launch finalize+apply (atomic statistics) parity, attention / int8 kernels,
# then the bench (bf16 headline + fp32 record), the step profile and the int8 VGG16 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
# test step: assertion failures (rc 1) are recorded and the script goes on; a crash, abort or time
# limit ends it
t() { local log=$1 lim=$2; shift 2; timeout -k 10 $lim $T "$@" > gpurun_out/r4c/$log 2>&1; local rc=$?
      tail -2 gpurun_out/r4c/$log; [ $rc -le 1 ] || exit $rc; }
t tests_bn.log 400 tests/test_resnet_block_parity.py tests/test_native_kernels.py tests/test_bn_prologue.py tests/test_syncbn_native.py
t tests_rnn.log 300 tests/test_rnn_persistent.py
for v in 0 2 3; do
  BIGDL_RNN_PERSIST=$v timeout -k 10 300 python tools/bench_configs.py --config ptb --steps 20 --warmup 5 > gpurun_out/r4c/ptb_p$v.log 2>&1 || { tail -30 gpurun_out/r4c/ptb_p$v.log; exit 1; }
  tail -1 gpurun_out/r4c/ptb_p$v.log
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4c/bench.log 2>&1 || { tail -30 gpurun_out/r4c/bench.log; exit 1; }
tail -1 gpurun_out/r4c/bench.log
t tests_attn.log 300 tests/test_attn_decode_native.py tests/test_attention_native.py tests/test_attention_module_native.py
t tests_i8.log 300 tests/test_conv_i8_native.py tests/test_quantized.py
timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r4c/int8.log 2>&1 || { tail -30 gpurun_out/r4c/int8.log; exit 1; }
tail -1 gpurun_out/r4c/int8.log
bash tools/prof_resnet.sh || exit 1
cp gpurun_out/prof_rn_summary.txt gpurun_out/r4c/
for v in 0 1; do
  BIGDL_CONV_X8=1 BIGDL_CONV_X8_ILV=$v timeout -k 10 300 python -u tools/pw_bench.py > gpurun_out/r4c/pw_x8_ilv$v.jsonl 2>&1 || { tail -20 gpurun_out/r4c/pw_x8_ilv$v.jsonl; exit 1; }
  tail -1 gpurun_out/r4c/pw_x8_ilv$v.jsonl
done
