#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5av
for i in 1 2 3; do
  for v in 1 0; do
    BIGDL_FUSION_SHORTCUTBN=$v timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5av/b${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5av/b${v}_$i.log; exit 1; }
    echo "shortcutbn=$v $i $(grep metric gpurun_out/r5av/b${v}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
BIGDL_FUSION_SHORTCUTBN=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_parity.py -k "local_vs_distri" > gpurun_out/r5av/t0.log 2>&1; echo "parity test with shortcutbn=0: rc=$?"; tail -1 gpurun_out/r5av/t0.log
