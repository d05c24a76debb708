#!/bin/bash
# early training curves: bf16 native, fp32 native (bf16x3 kernels), fp32 on torch/MIOpen (bigdl.fp32.native=false)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ah
mkdir -p $O
timeout -k 10 300 python -u tools/convergence.py --dtype bf16 --steps 300 --batch 128 --log-every 10 > $O/bf16.log 2>&1 || { tail -20 $O/bf16.log; exit 1; }
timeout -k 10 300 python -u tools/convergence.py --dtype fp32 --steps 300 --batch 128 --log-every 10 > $O/fp32.log 2>&1 || { tail -20 $O/fp32.log; exit 1; }
BIGDL_FP32_NATIVE=0 timeout -k 10 600 python -u tools/convergence.py --dtype fp32 --steps 300 --batch 128 --log-every 10 > $O/fp32_torch.log 2>&1 || { tail -20 $O/fp32_torch.log; exit 1; }
paste <(grep '"step"' $O/bf16.log | python3 -c 'import sys,json; [print(json.loads(l)["step"], json.loads(l)["loss"]) for l in sys.stdin]') <(grep '"step"' $O/fp32.log | python3 -c 'import sys,json; [print(json.loads(l)["loss"]) for l in sys.stdin]') <(grep '"step"' $O/fp32_torch.log | python3 -c 'import sys,json; [print(json.loads(l)["loss"]) for l in sys.stdin]')
