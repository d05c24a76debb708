#!/bin/bash
# DistriOptimizer world 1 with the shard tensors aliasing the arena (bigdl.comm.aliasWorld1): GPU
# distri tests; PTB and ResNet-50 local vs distri (alias) vs distri (no alias), interleaved repeats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distri_ptb.py tests/test_distri_resnet.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
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
