#!/bin/bash
# round 6 batch: new GPU tests (fp32 no-fallback, int8 residual), fp32 parity, int8 ResNet-50 bench,
# fp32 BN apply knobs, PTB distri world 1, fp32 config numbers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_int8_static.py tests/test_no_fallback.py tests/test_compiled.py tests/test_lstm_stack.py tests/test_fp32_direct.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u -m pytest -x -s -v --timeout 300 --timeout-method thread tests/test_train_parity.py -k fp32 > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
grep -A3 "fp32 ResNet-50" $O/parity.log; tail -1 $O/parity.log
timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model resnet50 --calib 32 --steps 20 --warmup 5 > $O/int8_resnet.log 2>&1 || { tail -30 $O/int8_resnet.log; exit 1; }
grep '^{' $O/int8_resnet.log | tail -1
for u in 4 8 2; do
  BIGDL_BN32_UNROLL=$u timeout -k 10 120 python tools/bench_bn32.py > $O/bn32_u$u.log 2>&1 || { tail -20 $O/bn32_u$u.log; exit 1; }
  tail -1 $O/bn32_u$u.log
done
for b in 1024 4096; do
  BIGDL_BN32_BLOCKS=$b timeout -k 10 120 python tools/bench_bn32.py > $O/bn32_b$b.log 2>&1 || { tail -20 $O/bn32_b$b.log; exit 1; }
  tail -1 $O/bn32_b$b.log
done
cat $O/bn32_u4.log | head -9
for i in 1 2; do
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 > $O/ptb_local_$i.log 2>&1 || { tail -20 $O/ptb_local_$i.log; exit 1; }
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --force-distri > $O/ptb_distri_$i.log 2>&1 || { tail -20 $O/ptb_distri_$i.log; exit 1; }
  grep -h '^{' $O/ptb_local_$i.log $O/ptb_distri_$i.log | python -c 'import json,sys; [print(d["config"].get("driver"), d["config"].get("update_mode"), d["ms_per_step"], d["value"]) for d in map(json.loads, sys.stdin)]'
done
for c in ptb vgg inception; do
  timeout -k 10 300 python tools/bench_configs.py --config $c --dtype fp32 > $O/${c}_fp32.log 2>&1 || { tail -20 $O/${c}_fp32.log; exit 1; }
  grep '^{' $O/${c}_fp32.log | tail -1 | cut -c1-400
done
