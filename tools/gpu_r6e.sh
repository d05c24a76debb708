#!/bin/bash
# fp32 step knob A/B: wgrad CU mask, BN apply grid cap (interleaved, 2 repeats)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 --phase-steps 0 > gpurun_out/r6e/$name.log 2>&1 || { tail -20 gpurun_out/r6e/$name.log; exit 1; }
  echo "$name $(grep metric gpurun_out/r6e/$name.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
for i in 1 2; do
  run base_$i BIGDL_X=0 || exit 1
  run cu34_$i BIGDL_WGRAD_CUMASK=3/4 || exit 1
  run cu12_$i BIGDL_WGRAD_CUMASK=1/2 || exit 1
  run apply1024_$i BIGDL_BN_APPLY_BLOCKS=1024 || exit 1
  run apply4096_$i BIGDL_BN_APPLY_BLOCKS=4096 || exit 1
  run noasync_$i BIGDL_CONV_ASYNCWGRAD=0 || exit 1
done
bash tools/prof_fp32.sh > /dev/null && cp gpurun_out/prof_f32_summary.txt gpurun_out/r6e/ && head -45 gpurun_out/r6e/prof_f32_summary.txt
