#!/bin/bash
# VGG-CIFAR / Inception-v1 regression check: round-3 tree (ab_r3, commit b385f3c) vs HEAD, interleaved, 3 repeats
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6q
mkdir -p $O
for i in 1 2 3; do
  for tree in r3 head; do
    d=.; [ $tree = r3 ] && d=ab_r3
    (cd $d && timeout -k 10 200 python tools/bench_configs.py --config vgg > $O/vgg_${tree}_$i.log 2>&1) || { tail -20 $O/vgg_${tree}_$i.log; exit 1; }
    echo "vgg $tree $i $(grep '^{' $O/vgg_${tree}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
    (cd $d && timeout -k 10 300 python tools/bench_configs.py --config inception > $O/inc_${tree}_$i.log 2>&1) || { tail -20 $O/inc_${tree}_$i.log; exit 1; }
    echo "inception $tree $i $(grep '^{' $O/inc_${tree}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
