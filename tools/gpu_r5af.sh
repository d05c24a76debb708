#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5af
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_patch.py tests/test_conv_x8.py > gpurun_out/r5af/test.log 2>&1 || { tail -40 gpurun_out/r5af/test.log; exit 1; }
tail -1 gpurun_out/r5af/test.log
for v in 1 0; do
  BIGDL_CONV_PATCH=$v ONLY3=1 timeout -k 10 300 python tools/pw_bench.py > gpurun_out/r5af/pw3_patch$v.jsonl 2>&1 || { tail -20 gpurun_out/r5af/pw3_patch$v.jsonl; exit 1; }
  echo "patch=$v $(grep '"C": 64, "K": 64, "R": 3' gpurun_out/r5af/pw3_patch$v.jsonl | cut -c40-140)"
done



