#!/bin/bash
# kernel stats of the int8 VGG16 run with unsigned activations on / off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5x
for u in 1 0; do
  BIGDL_INT8_UNSIGNEDACTIVATIONS=$u timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5x/p$u -o run -- python3 tools/bench_configs.py --config int8 --steps 5 --warmup 2 --calib 64 > gpurun_out/r5x/u$u.log 2>&1 || { tail -20 gpurun_out/r5x/u$u.log; exit 1; }
  db=$(find gpurun_out/r5x/p$u -name '*.db' | head -1)
  python3 tools/rocpd_summary.py "$db" 1 40 > gpurun_out/r5x/sum_u$u.txt
  python3 tools/rocpd_dispatches.py "$db" 400 > gpurun_out/r5x/disp_u$u.txt; rm -rf gpurun_out/r5x/p$u
done
grep -i "conv_i8\|quant\|maxpool" gpurun_out/r5x/sum_u1.txt gpurun_out/r5x/sum_u0.txt
