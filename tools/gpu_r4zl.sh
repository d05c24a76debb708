#!/bin/bash
# World-1 A/B on one box: local vs --force-distri --syncbn (SyncBN kernels, collectives skipped) vs --force-distri bf16 wire
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zl
run() { timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --phase-steps 0 "$@" > gpurun_out/r4zl/$1$2.log 2>&1 || { tail -20 gpurun_out/r4zl/$1$2.log; return 1; }; tail -1 gpurun_out/r4zl/$1$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
echo "local $(run)" && echo "syncbn $(run --force-distri --syncbn)" && echo "distri $(run --force-distri --comm-dtype bf16)" && echo "local $(run)"
