#!/bin/bash
# SyncBN kernel tests + syncbn vs syncmr kernel summaries; int8 ResNet-50 / Inception with the short-K
# default and the int8 FC head; PTB world 1 local vs distri (3 interleaved repeats)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_syncbn_native.py tests/test_int8_fc.py tests/test_conv_i8_native.py tests/test_int8_static.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
for cfg in syncbn syncmr; do
  e=""; [ $cfg = syncmr ] && e="BIGDL_BN_SYNCONERANKLOCAL=0"
  env $e timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p_$cfg -o run -- python3 bench.py --steps 5 --warmup 3 --fp32-steps 0 --force-distri --syncbn > $O/p_$cfg.log 2>&1 || { tail -20 $O/p_$cfg.log; exit 1; }
  db=$(find $O/p_$cfg -name '*.db' | head -1)
  LAST_MS=110 python3 tools/rocpd_summary.py $db 5 60 > $O/k_$cfg.txt
  head -3 $O/k_$cfg.txt
  rm -rf $O/p_$cfg
done
for mdl in resnet50 inception; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 20 --warmup 5 > $O/int8_$mdl.log 2>&1 || { tail -30 $O/int8_$mdl.log; exit 1; }
  grep '^{' $O/int8_$mdl.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], "int8", d["ms_per_step"], "graph", d.get("int8_graph"), "bf16c", d.get("bf16_compiled"), "cos", d["cosine_int8_vs_fp32"], "fc", d["fc_dtype"])'
done
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 > $O/ptb_local_$i.log 2>&1 || { tail -20 $O/ptb_local_$i.log; exit 1; }
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --force-distri > $O/ptb_distri_$i.log 2>&1 || { tail -20 $O/ptb_distri_$i.log; exit 1; }
  grep -h '^{' $O/ptb_local_$i.log $O/ptb_distri_$i.log | python -c 'import json,sys; [print(d["config"].get("driver"), d["ms_per_step"], d["value"]) for d in map(json.loads, sys.stdin)]'
done
