#!/bin/bash
# repeat the harder-task curves (700 steps): bf16, fp32 native, fp32 native without the BN prologue, fp32 torch/MIOpen
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6aj
mkdir -p $O
A="--steps 700 --batch 128 --classes 1000 --noise 2 --log-every 50"
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/convergence.py --dtype bf16 $A > $O/bf16_$i.log 2>&1 || { tail -20 $O/bf16_$i.log; exit 1; }
  timeout -k 10 200 python -u tools/convergence.py --dtype fp32 $A > $O/fp32_$i.log 2>&1 || { tail -20 $O/fp32_$i.log; exit 1; }
  BIGDL_FP32_BNPROLOGUE=0 timeout -k 10 200 python -u tools/convergence.py --dtype fp32 $A > $O/fp32np_$i.log 2>&1 || { tail -20 $O/fp32np_$i.log; exit 1; }
  BIGDL_FP32_NATIVE=0 timeout -k 10 400 python -u tools/convergence.py --dtype fp32 $A > $O/fp32t_$i.log 2>&1 || { tail -20 $O/fp32t_$i.log; exit 1; }
  for a in bf16 fp32 fp32np fp32t; do
    echo "$a $i $(grep '"step"' $O/${a}_$i.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["loss"]) for l in sys.stdin))') acc $(grep final $O/${a}_$i.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["heldout_acc"])')"
  done
done
