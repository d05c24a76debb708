#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for sh in 64,256,1,1,56 256,1024,1,1,14 64,64,3,1,56 256,64,1,1,56; do
  timeout -k 10 120 python -u tools/bench_x3.py --only $sh --out /tmp/a.jsonl 2>&1 | grep -v amdgpu.ids
done
