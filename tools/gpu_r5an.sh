#!/bin/bash
# bf16 step knob sweep, interleaved, 3 repeats per arm
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5an
ARMS=("base:" "fold:BIGDL_BN_FOLDFINALIZE=1" "ilv0:BIGDL_CONV_X8_ILV=0" "wepi1:BIGDL_WGRAD_EPI=1" "wfirst0:BIGDL_WGRAD_FIRST=0")
for i in 1 2 3; do
  for a in "${ARMS[@]}"; do
    name=${a%%:*}; kv=${a#*:}
    env $kv timeout -k 10 400 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r5an/${name}_$i.log 2>&1 || { tail -20 gpurun_out/r5an/${name}_$i.log; exit 1; }
    echo "$name $i $(grep metric gpurun_out/r5an/${name}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
