#!/bin/bash
# PTB LSTM LM training curves on a learnable Markov-chain language: bf16 native, fp32 native, fp32 torch; 2 repeats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6au
mkdir -p $O
for i in 1 2; do
  for arm in bf16 fp32 fp32t; do
    case $arm in bf16) e=""; d=bf16;; fp32) e=""; d=fp32;; fp32t) e="BIGDL_FP32_NATIVE=0"; d=fp32;; esac
    env $e timeout -k 10 500 python -u tools/convergence_ptb.py --dtype $d --steps 2000 --log-every 200 > $O/${arm}_$i.log 2>&1 || { tail -20 $O/${arm}_$i.log; exit 1; }
    echo "$arm $i $(grep '"step"' $O/${arm}_$i.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["nats_per_token"]) for l in sys.stdin))') $(grep final $O/${arm}_$i.log | cut -c1-160)"
  done
done
for i in 1 2; do
  for arm in bf16 fp32 fp32t; do
    case $arm in bf16) e=""; d=bf16;; fp32) e=""; d=fp32;; fp32t) e="BIGDL_FP32_NATIVE=0"; d=fp32;; esac
    env $e timeout -k 10 300 python -u tools/convergence.py --model vgg_cifar --dtype $d --steps 2000 --batch 128 --classes 100 --noise 2 --lr 0.05 --log-every 200 > $O/vgg_${arm}_$i.log 2>&1 || { tail -20 $O/vgg_${arm}_$i.log; exit 1; }
    echo "vgg $arm $i $(grep '"step"' $O/vgg_${arm}_$i.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["loss"]) for l in sys.stdin))') acc $(grep final $O/vgg_${arm}_$i.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["heldout_acc"])')"
  done
done
