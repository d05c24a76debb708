#!/bin/bash
# round 6 batch: fp32 trajectory parity, int8 ResNet-50 / Inception vs compiled bf16, PTB distri world 1
# (sharded Adagrad), fp32 config numbers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -s -v --timeout 300 --timeout-method thread tests/test_train_parity.py -k fp32 > $O/parity.log 2>&1; rc=$?
grep -A3 "fp32 ResNet-50" $O/parity.log; tail -1 $O/parity.log
[ $rc -le 1 ] || exit 1
for mdl in resnet50 inception; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 20 --warmup 5 > $O/int8_$mdl.log 2>&1 || { tail -30 $O/int8_$mdl.log; exit 1; }
  grep '^{' $O/int8_$mdl.log | tail -1
done
for i in 1 2; do
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 > $O/ptb_local_$i.log 2>&1 || { tail -20 $O/ptb_local_$i.log; exit 1; }
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --force-distri > $O/ptb_distri_$i.log 2>&1 || { tail -20 $O/ptb_distri_$i.log; exit 1; }
  grep -h '^{' $O/ptb_local_$i.log $O/ptb_distri_$i.log | python -c 'import json,sys; [print(d["config"].get("driver"), d["config"].get("update_mode"), d["ms_per_step"], d["value"]) for d in map(json.loads, sys.stdin)]'
done
for c in ptb vgg inception lenet; do
  timeout -k 10 300 python tools/bench_configs.py --config $c --dtype fp32 > $O/${c}_fp32.log 2>&1 || { tail -20 $O/${c}_fp32.log; exit 1; }
  grep '^{' $O/${c}_fp32.log | tail -1 | cut -c1-600
done
