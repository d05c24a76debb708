#!/bin/bash
# SyncBN multi-rank kernels with the projection-shortcut deferral: tests + 3 interleaved repeats of
# local BN / forced-distri one-rank-local SyncBN / forced-distri multi-rank SyncBN kernels (bf16 bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_syncbn_native.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for cfg in local syncbn syncmr; do
    case $cfg in local) a=""; e="";; syncbn) a="--force-distri --syncbn"; e="";; syncmr) a="--force-distri --syncbn"; e="BIGDL_BN_SYNCONERANKLOCAL=0";; esac
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 $a > $O/${cfg}_$i.log 2>&1 || { tail -20 $O/${cfg}_$i.log; exit 1; }
    echo "$cfg $i $(grep metric $O/${cfg}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
