#!/bin/bash
# Round 4 (i): launch lag in the ResNet-50 step; 16-B granule loads in the 4-wave LSTM; int8 test.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_rnn_persistent.py -k "6 or 7" > gpurun_out/r4i/tests_rnn.log 2>&1; rc=$?
tail -3 gpurun_out/r4i/tests_rnn.log; [ $rc -le 1 ] || exit $rc
if [ $rc -eq 0 ]; then
for v in 0 6 7; do
  BIGDL_RNN_PERSIST=$v timeout -k 10 300 python tools/bench_configs.py --config ptb --steps 20 --warmup 5 > gpurun_out/r4i/ptb_p$v.log 2>&1 || { tail -30 gpurun_out/r4i/ptb_p$v.log; exit 1; }
  tail -1 gpurun_out/r4i/ptb_p$v.log | cut -c1-160
done
fi
timeout -k 10 300 $T tests/test_conv_i8_native.py > gpurun_out/r4i/tests_i8.log 2>&1; rc=$?
tail -3 gpurun_out/r4i/tests_i8.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r4i/lag -o run -- python bench.py --steps 3 --warmup 3 --phase-steps 0 --fp32-steps 0 > gpurun_out/r4i/lag.log 2>&1 || { tail -20 gpurun_out/r4i/lag.log; exit 1; }
db=$(find gpurun_out/r4i/lag -name '*.db' | head -1)
ms=$(python -c "import json; print([json.loads(l) for l in open('gpurun_out/r4i/lag.log') if l.startswith('{\"metric')][-1]['ms_per_step'])")
python tools/launch_lag.py "$db" $ms 2 > gpurun_out/r4i/lag_summary.txt 2>&1
cp "$db" gpurun_out/r4i/lag.db 2>/dev/null; rm -rf gpurun_out/r4i/lag
head -40 gpurun_out/r4i/lag_summary.txt
