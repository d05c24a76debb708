#!/bin/bash
# Round 4 (g): 4-wave granule LSTM (modes 6/7) tests + PTB A/B, host enqueue profile, the distri /
# SyncBN world-1 rehearsals.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_rnn_persistent.py -k "6 or 7" > gpurun_out/r4g/tests_rnn.log 2>&1; rc=$?
tail -3 gpurun_out/r4g/tests_rnn.log; [ $rc -le 1 ] || exit $rc
if [ $rc -eq 0 ]; then
for v in 0 6 7; do
  BIGDL_RNN_PERSIST=$v timeout -k 10 300 python tools/bench_configs.py --config ptb --steps 20 --warmup 5 > gpurun_out/r4g/ptb_p$v.log 2>&1 || { tail -30 gpurun_out/r4g/ptb_p$v.log; exit 1; }
  tail -1 gpurun_out/r4g/ptb_p$v.log | cut -c1-160
done
fi
bash tools/gpu_r4f.sh
