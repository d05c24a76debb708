#!/bin/bash
# Validation after moving the tile choice into the launch: full GPU suite + bench, VGG tuned eager/graph.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3i
PROFILE=0 bash tools/gpu_check.sh || exit 1
for a in "--tune" "--graph --tune"; do
  timeout -k 10 240 python tools/bench_configs.py --config vgg --steps 30 --warmup 5 $a > gpurun_out/r3i/vgg.log 2>&1 || { tail -20 gpurun_out/r3i/vgg.log; exit 1; }
  echo "args=[$a] $(grep '^{' gpurun_out/r3i/vgg.log | tail -1)"
done
