#!/bin/bash
# Round 4 (e): fixed tests, stats-epilogue cost per shape (+ kernel names), bench with the x8
# interleaved-DMA default, int8 VGG16 with data-dependent init.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
t() { local log=$1 lim=$2; shift 2; timeout -k 10 $lim $T "$@" > gpurun_out/r4e/$log 2>&1; local rc=$?
      tail -2 gpurun_out/r4e/$log; [ $rc -le 1 ] || exit $rc; }
t tests_fix.log 300 tests/test_native_kernels.py tests/test_bn_prologue.py tests/test_resnet_block_parity.py tests/test_graph_adam.py tests/test_conv_i8_native.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/st -o run -- python tools/stats_ab.py > gpurun_out/r4e/stats_ab.log 2>&1 || { tail -30 gpurun_out/r4e/stats_ab.log; exit 1; }
grep '^{' gpurun_out/r4e/stats_ab.log
db=$(find gpurun_out/r4e/st -name '*.db' | head -1)
python tools/rocpd_summary.py "$db" 1 40 > gpurun_out/r4e/stats_ab_kernels.txt; rm -rf gpurun_out/r4e/st
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4e/bench.log 2>&1 || { tail -30 gpurun_out/r4e/bench.log; exit 1; }
tail -1 gpurun_out/r4e/bench.log | cut -c1-250
timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r4e/int8.log 2>&1 || { tail -30 gpurun_out/r4e/int8.log; exit 1; }
tail -1 gpurun_out/r4e/int8.log
t tests_rnn.log 400 tests/test_rnn_persistent.py
for v in 0 4 5 6 7; do
  BIGDL_RNN_PERSIST=$v timeout -k 10 300 python tools/bench_configs.py --config ptb --steps 20 --warmup 5 > gpurun_out/r4e/ptb_p$v.log 2>&1 || { tail -30 gpurun_out/r4e/ptb_p$v.log; exit 1; }
  tail -1 gpurun_out/r4e/ptb_p$v.log | cut -c1-160
done
for cfg in BIGDL_DEBUG_WGRAD_NO_ATOMICS=1 BIGDL_WGRAD_EPI=1 BIGDL_FUSION_BNPROLOGUE=2 BIGDL_CONV_X8_ILV=0; do
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4e/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/r4e/bench_$cfg.log; exit 1; }
  echo "$cfg"; tail -1 gpurun_out/r4e/bench_$cfg.log | cut -c1-200
done
bash tools/prof_timeline.sh r4tl --fp32-steps 0 || exit 1
cp gpurun_out/prof_r4tl_summary.txt gpurun_out/prof_r4tl_timeline.txt gpurun_out/r4e/ && rm -f gpurun_out/prof_r4tl.db
