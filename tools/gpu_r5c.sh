#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 400 python -u tools/bench_x3.py --out gpurun_out/r5c/bench_x3.jsonl 2>&1 | tee gpurun_out/r5c/bench_x3.log
