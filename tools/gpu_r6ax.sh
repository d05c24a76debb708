#!/bin/bash
# Re-entry check on a fresh box: the full GPU suite, the driver's bench line, then the world-1
# DistriOptimizer shard-alias A/B (bigdl.comm.aliasWorld1) on PTB and ResNet-50, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ax
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then grep -v INFO $O/pytest_gpu.log | tail -40; exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], "fp32", d["fp32"]["ms_per_step"])'
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 > $O/ptb_local_$i.log 2>&1 || { tail -20 $O/ptb_local_$i.log; exit 1; }
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --force-distri > $O/ptb_alias_$i.log 2>&1 || { tail -20 $O/ptb_alias_$i.log; exit 1; }
  BIGDL_COMM_ALIASWORLD1=0 timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --force-distri > $O/ptb_noalias_$i.log 2>&1 || { tail -20 $O/ptb_noalias_$i.log; exit 1; }
  for k in local alias noalias; do echo -n "ptb $k "; grep -h '^{' $O/ptb_${k}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"].get("driver"), d["ms_per_step"], d["value"])'; done
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 --fp32-steps 0 > $O/rn_local_$i.log 2>&1 || { tail -20 $O/rn_local_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 --fp32-steps 0 --force-distri > $O/rn_alias_$i.log 2>&1 || { tail -20 $O/rn_alias_$i.log; exit 1; }
  BIGDL_COMM_ALIASWORLD1=0 timeout -k 10 300 python bench.py --steps 30 --warmup 8 --fp32-steps 0 --force-distri > $O/rn_noalias_$i.log 2>&1 || { tail -20 $O/rn_noalias_$i.log; exit 1; }
  for k in local alias noalias; do echo -n "resnet50 $k "; grep -h '^{' $O/rn_${k}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; done
done
