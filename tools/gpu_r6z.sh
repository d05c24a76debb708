#!/bin/bash
# new tests (int8 FC head, SyncBN deferral), int8 short-K tile variants, int8 FC on/off, then the
# SyncBN A/B (tools/gpu_r6y.sh) and the PTB world-1 host profile (tools/gpu_r6x.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_int8_fc.py tests/test_syncbn_native.py tests/test_fp32_bn_prologue.py > $O/new_tests.log 2>&1 || { grep -v INFO $O/new_tests.log | tail -40; exit 1; }
tail -1 $O/new_tests.log
timeout -k 10 200 python tools/i8_shortk_bench.py > $O/shortk.log 2>&1 || { tail -20 $O/shortk.log; exit 1; }
cat $O/shortk.log
for fc in 0 1; do
  timeout -k 10 300 python tools/bench_configs.py --config int8 --calib 32 --steps 20 --warmup 5 --int8-fc $fc > $O/vgg_fc$fc.log 2>&1 || { tail -30 $O/vgg_fc$fc.log; exit 1; }
  grep '^{' $O/vgg_fc$fc.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("vgg16 fc", d["fc_dtype"], d["ms_per_step"], d["value"], "cos", d["cosine_int8_vs_fp32"], "top1", d["top1_agreement"], "bf16", d["bf16"])'
done
bash tools/gpu_r6y.sh && bash tools/gpu_r6x.sh
