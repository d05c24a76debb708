#!/bin/bash
# fp32 native training instability: weight gradients inline (BIGDL_CONV_ASYNCWGRAD=0) vs forked onto the side stream
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6al
mkdir -p $O
A="--steps 700 --batch 128 --classes 1000 --noise 2 --log-every 50"
for i in 1 2 3; do
  for arm in inline async; do
    e=""; [ $arm = inline ] && e="BIGDL_CONV_ASYNCWGRAD=0"
    env $e timeout -k 10 200 python -u tools/convergence.py --dtype fp32 $A > $O/${arm}_$i.log 2>&1 || { tail -20 $O/${arm}_$i.log; exit 1; }
    echo "$arm $i $(grep '"step"' $O/${arm}_$i.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["loss"]) for l in sys.stdin))') acc $(grep final $O/${arm}_$i.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["heldout_acc"])')"
  done
done
