#!/bin/bash
# Secondary BASELINE configs at the reference's precision (fp32 compute), 3 repeats each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6bf
mkdir -p $O
for i in 1 2 3; do
  for c in vgg ptb inception; do
    timeout -k 10 300 python tools/bench_configs.py --config $c --dtype fp32 > $O/${c}_$i.log 2>&1 || { tail -30 $O/${c}_$i.log; exit 1; }
    grep -h '^{' $O/${c}_$i.log | tail -1 >> $O/fp32_configs.jsonl
    grep -h '^{' $O/${c}_$i.log | tail -1 | cut -c1-400
    grep -hi "fell back" $O/${c}_$i.log | head -3 || true
  done
done
