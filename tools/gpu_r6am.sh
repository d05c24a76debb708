#!/bin/bash
# which fp32-native component destabilises training: toggles of the fp32 fusions (2 repeats each)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6am
mkdir -p $O
A="--steps 600 --batch 128 --classes 1000 --noise 2 --log-every 50"
for i in 1 2; do
  for arm in convstats0 direct0 stemc40 det1; do
    case $arm in convstats0) e="BIGDL_FP32_CONVSTATS=0";; direct0) e="BIGDL_FP32_DIRECT=0";; stemc40) e="BIGDL_FP32_STEMC4=0";; det1) e="BIGDL_DETERMINISTIC=1";; esac
    env $e timeout -k 10 200 python -u tools/convergence.py --dtype fp32 $A > $O/${arm}_$i.log 2>&1 || { tail -20 $O/${arm}_$i.log; exit 1; }
    echo "$arm $i $(grep '"step"' $O/${arm}_$i.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["loss"]) for l in sys.stdin))') acc $(grep final $O/${arm}_$i.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["heldout_acc"])')"
  done
done
