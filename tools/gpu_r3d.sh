#!/bin/bash
# Full GPU suite + ResNet-50 bench + kernel profile + smoke, then the Inception-v1 inference config
# (32-bit index inference max-pool).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
PROFILE=0 bash tools/gpu_check.sh || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d/smoke.log 2>&1 || { tail -20 gpurun_out/r3d/smoke.log; exit 1; }
tail -1 gpurun_out/r3d/smoke.log
bash tools/prof_resnet.sh || exit 1
timeout -k 10 300 python tools/bench_configs.py --config inception --steps 30 --warmup 5 > gpurun_out/r3d/inception.log 2>&1 || { tail -20 gpurun_out/r3d/inception.log; exit 1; }
tail -1 gpurun_out/r3d/inception.log
