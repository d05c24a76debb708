#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5k
timeout -k 10 400 python -u tools/pw_bench.py > gpurun_out/r5k/pw.jsonl 2>&1 || { tail -5 gpurun_out/r5k/pw.jsonl; exit 1; }
cat gpurun_out/r5k/pw.jsonl | cut -c1-330
