#!/bin/bash
# int8 on a trained ResNet-50 (synthetic task), partially trained / noisier so top-1 is not saturated
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6av
mkdir -p $O
for cfg in "300 4" "600 8" "1500 12"; do
  set -- $cfg
  timeout -k 10 600 python -u tools/int8_trained.py --steps $1 --classes 1000 --noise $2 > $O/trained_$1_$2.log 2>&1 || { tail -30 $O/trained_$1_$2.log; exit 1; }
  grep final $O/trained_$1_$2.log
done
