#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6o
timeout -k 10 300 python tools/pro_diag.py > gpurun_out/r6o/diag.log 2>&1 || { tail -30 gpurun_out/r6o/diag.log; exit 1; }
grep -v "INFO bigdl" gpurun_out/r6o/diag.log | head -300
