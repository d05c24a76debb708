#!/bin/bash
# harder synthetic task (1000 classes, noise 2): bf16 native vs fp32 native (1500 steps) vs fp32 torch/MIOpen (600 steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 300 python -u tools/convergence.py --dtype bf16 --steps 1500 --batch 128 --classes 1000 --noise 2 --log-every 50 > $O/bf16.log 2>&1 || { tail -20 $O/bf16.log; exit 1; }
timeout -k 10 400 python -u tools/convergence.py --dtype fp32 --steps 1500 --batch 128 --classes 1000 --noise 2 --log-every 50 > $O/fp32.log 2>&1 || { tail -20 $O/fp32.log; exit 1; }
BIGDL_FP32_NATIVE=0 timeout -k 10 600 python -u tools/convergence.py --dtype fp32 --steps 600 --batch 128 --classes 1000 --noise 2 --log-every 50 > $O/fp32_torch.log 2>&1 || { tail -20 $O/fp32_torch.log; exit 1; }
for f in bf16 fp32 fp32_torch; do grep final $O/$f.log; done
