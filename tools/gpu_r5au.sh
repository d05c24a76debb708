#!/bin/bash
# deferred shortcut BN: full GPU suite, then bench shortcutbn on / off interleaved (3 repeats)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5au
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5au/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r5au/gpu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5au/gpu_tests.log | tail -1
for i in 1 2 3; do
  for v in 1 0; do
    BIGDL_FUSION_SHORTCUTBN=$v timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5au/b${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5au/b${v}_$i.log; exit 1; }
    echo "shortcutbn=$v $i $(grep metric gpurun_out/r5au/b${v}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
