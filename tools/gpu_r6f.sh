#!/bin/bash
# round 6: fp32 no-fallback tests (LeNet / PTB / Inception), PTB distri world-1, fp32 config numbers
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6f
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_no_fallback.py tests/test_lstm_stack.py tests/test_compiled.py > gpurun_out/r6f/tests.log 2>&1 || { tail -40 gpurun_out/r6f/tests.log; exit 1; }
tail -3 gpurun_out/r6f/tests.log
timeout -k 10 400 python -u -m pytest -x -s -v --timeout 300 --timeout-method thread tests/test_train_parity.py -k fp32 > gpurun_out/r6f/parity.log 2>&1 || { tail -40 gpurun_out/r6f/parity.log; exit 1; }
grep -A3 "fp32 ResNet-50" gpurun_out/r6f/parity.log; tail -2 gpurun_out/r6f/parity.log
for i in 1 2; do
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 > gpurun_out/r6f/ptb_local_$i.log 2>&1 || { tail -20 gpurun_out/r6f/ptb_local_$i.log; exit 1; }
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --force-distri > gpurun_out/r6f/ptb_distri_$i.log 2>&1 || { tail -20 gpurun_out/r6f/ptb_distri_$i.log; exit 1; }
  grep '^{' gpurun_out/r6f/ptb_local_$i.log | tail -1
  grep '^{' gpurun_out/r6f/ptb_distri_$i.log | tail -1
  grep -h "mode=" gpurun_out/r6f/ptb_distri_$i.log | tail -1
done
for c in ptb vgg inception; do
  timeout -k 10 300 python tools/bench_configs.py --config $c --dtype fp32 > gpurun_out/r6f/${c}_fp32.log 2>&1 || { tail -20 gpurun_out/r6f/${c}_fp32.log; exit 1; }
  grep '^{' gpurun_out/r6f/${c}_fp32.log | tail -1
done
