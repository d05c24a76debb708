#!/bin/bash
# end-of-round evidence: fp32 bench, SyncBN world-1 A/B, compiled inference, PTB — 3 repeats each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5al
J='import json,sys; d=[json.loads(l) for l in sys.stdin if l.startswith("{\"metric")][-1]'
for i in 1 2 3; do
  timeout -k 10 500 python bench.py --steps 5 --warmup 3 --fp32-steps 10 > gpurun_out/r5al/fp32_$i.log 2>&1 || { tail -20 gpurun_out/r5al/fp32_$i.log; exit 1; }
  echo "fp32 $i $(python -c "$J; print(d['fp32']['ms_per_step'], d['fp32']['value'], d['ms_per_step'])" < gpurun_out/r5al/fp32_$i.log)"
done
for i in 1 2 3; do
  for arm in local syncbn; do
    A=""; [ $arm = syncbn ] && A="--force-distri --syncbn"
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 $A > gpurun_out/r5al/${arm}_$i.log 2>&1 || { tail -20 gpurun_out/r5al/${arm}_$i.log; exit 1; }
    echo "$arm $i $(python -c "$J; print(d['ms_per_step'], d['value'])" < gpurun_out/r5al/${arm}_$i.log)"
  done
done
for i in 1 2 3; do
  BATCHES=1,256 timeout -k 10 400 python tools/bench_infer.py > gpurun_out/r5al/infer_$i.log 2>&1 || { tail -20 gpurun_out/r5al/infer_$i.log; exit 1; }
  echo "infer $i $(grep -h '"batch"' gpurun_out/r5al/infer_$i.log | tr '\n' ' ' | cut -c1-400)"
done
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py --config ptb > gpurun_out/r5al/ptb_$i.log 2>&1 || { tail -20 gpurun_out/r5al/ptb_$i.log; exit 1; }
  echo "ptb $i $(python -c "$J; print(d['value'], d['ms_per_step'])" < gpurun_out/r5al/ptb_$i.log)"
done
