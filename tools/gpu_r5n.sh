#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5n
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --force-distri > gpurun_out/r5n/bench_distri_$rep.log 2>&1 || { tail -30 gpurun_out/r5n/bench_distri_$rep.log; exit 1; }
  echo "distri $rep $(tail -1 gpurun_out/r5n/bench_distri_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
BARGS="--force-distri --syncbn" bash tools/prof_resnet.sh > /dev/null && cp gpurun_out/prof_rn_summary.txt gpurun_out/r5n/prof_syncbn.txt
BARGS="--force-distri" bash tools/prof_resnet.sh > /dev/null && cp gpurun_out/prof_rn_summary.txt gpurun_out/r5n/prof_distri.txt
head -45 gpurun_out/r5n/prof_syncbn.txt
