#!/bin/bash
# Round 4 (f): host enqueue cost, the DistriOptimizer / SyncBN world-1 rehearsals against the local
# bench (verdict items 4 and 9), PTB granule A/B repeat.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
timeout -k 10 300 python tools/host_profile.py --batch 16 --steps 10 --big 256 --top 30 > gpurun_out/r4g/host.log 2>&1 || { tail -30 gpurun_out/r4g/host.log; exit 1; }
grep -i "enqueue\|step" gpurun_out/r4g/host.log | head -8
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4g/bench_local.log 2>&1 || { tail -30 gpurun_out/r4g/bench_local.log; exit 1; }
tail -1 gpurun_out/r4g/bench_local.log | cut -c1-220
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --force-distri --comm-dtype bf16 > gpurun_out/r4g/bench_distri_bf16.log 2>&1 || { tail -30 gpurun_out/r4g/bench_distri_bf16.log; exit 1; }
tail -1 gpurun_out/r4g/bench_distri_bf16.log | cut -c1-220
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 --force-distri --syncbn > gpurun_out/r4g/bench_syncbn.log 2>&1 || { tail -30 gpurun_out/r4g/bench_syncbn.log; exit 1; }
tail -1 gpurun_out/r4g/bench_syncbn.log | cut -c1-220
