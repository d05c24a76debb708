#!/bin/bash
# Round-3 re-entry: GPU tests + bench + kernel-stat profile + smoke, then wgrad-stream CU-mask A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
PROFILE=0 bash tools/gpu_check.sh || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b/smoke.log 2>&1 || { tail -20 gpurun_out/r3b/smoke.log; exit 1; }
tail -1 gpurun_out/r3b/smoke.log
bash tools/prof_resnet.sh || exit 1
for m in 3/4 1/2 none 7/8; do
  if [ "$m" = none ]; then unset BIGDL_WGRAD_CUMASK; else export BIGDL_WGRAD_CUMASK=$m; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/r3b/ab_${m/\//_}.log 2>&1 || { tail -20 gpurun_out/r3b/ab_${m/\//_}.log; exit 1; }
  echo "cumask=$m $(tail -1 gpurun_out/r3b/ab_${m/\//_}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
