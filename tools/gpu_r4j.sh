#!/bin/bash
# Round 4 (j): replicated atomic BN statistics (tests + A/B), SyncBN tail bits, wgrad-first fork,
# int8 VGG16 test, PTB kernel profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4j
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
t() { local log=$1 lim=$2; shift 2; timeout -k 10 $lim $T "$@" > gpurun_out/r4j/$log 2>&1; local rc=$?
      grep -E "^E  |passed|failed" gpurun_out/r4j/$log | head -12; [ $rc -le 1 ] || exit $rc; }
t tests_bn.log 400 tests/test_resnet_block_parity.py tests/test_native_kernels.py tests/test_bn_prologue.py tests/test_syncbn_native.py
t tests_i8.log 300 tests/test_conv_i8_native.py -k vgg16
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 $BARGS > gpurun_out/r4j/bench_$tag.log 2>&1 || { tail -30 gpurun_out/r4j/bench_$tag.log; exit 1; }
      echo "$tag $(tail -1 gpurun_out/r4j/bench_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; }
b base X=0
b rep64 BIGDL_BN_STATREPLICAS=64
b rep16 BIGDL_BN_STATREPLICAS=16
b wgfirst BIGDL_WGRAD_FIRST=1
BARGS="--force-distri --syncbn" b syncbn X=0
bash tools/gpu_r4k.sh || exit 1
