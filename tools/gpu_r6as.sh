#!/bin/bash
# fp32 BN apply knobs on the whole fp32 ResNet-50 step (3 interleaved repeats): rows in flight per thread, grid cap
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6as2
mkdir -p $O
for i in 1 2 3; do
  for arm in base u2 u1 u2b1024; do
    case $arm in base) e="";; u8) e="BIGDL_BN32_UNROLL=8";; u2) e="BIGDL_BN32_UNROLL=2";; b1024) e="BIGDL_BN32_BLOCKS=1024";; b4096) e="BIGDL_BN32_BLOCKS=4096";; u1) e="BIGDL_BN32_UNROLL=1";; u2b1024) e="BIGDL_BN32_UNROLL=2 BIGDL_BN32_BLOCKS=1024";; esac
    env $e timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > $O/${arm}_$i.log 2>&1 || { tail -20 $O/${arm}_$i.log; exit 1; }
    echo "$arm $i $(grep metric $O/${arm}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
