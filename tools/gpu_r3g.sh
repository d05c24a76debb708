#!/bin/bash
# Final validation: full GPU suite + smoke + ResNet-50 bench, then Inception eager vs compiled.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3g
PROFILE=0 bash tools/gpu_check.sh || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g/smoke.log 2>&1 || { tail -20 gpurun_out/r3g/smoke.log; exit 1; }
tail -1 gpurun_out/r3g/smoke.log
timeout -k 10 300 python tools/bench_configs.py --config inception --steps 30 --warmup 5 > gpurun_out/r3g/inc_eager.log 2>&1 || { tail -20 gpurun_out/r3g/inc_eager.log; exit 1; }
tail -1 gpurun_out/r3g/inc_eager.log
timeout -k 10 300 python tools/bench_configs.py --config inception --compiled --steps 30 --warmup 5 > gpurun_out/r3g/inc_comp.log 2>&1 || { tail -20 gpurun_out/r3g/inc_comp.log; exit 1; }
tail -1 gpurun_out/r3g/inc_comp.log
