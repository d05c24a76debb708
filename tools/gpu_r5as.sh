#!/bin/bash
# every BASELINE config once more at round end (+ VGG with graph/tuning), one JSON line each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5as
for c in "vgg" "vgg --graph --tune" "inception" "inception --compiled" "lenet" "transformer" "resnet_infer"; do
  n=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 500 python tools/bench_configs.py --config $c > gpurun_out/r5as/$n.log 2>&1 || { tail -20 gpurun_out/r5as/$n.log; exit 1; }
  echo "$c: $(grep '^{' gpurun_out/r5as/$n.log | tail -1 | cut -c1-300)"
done
