#!/bin/bash
# full GPU suite (incl. the 2-rank device rehearsal) + smoke + default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6be
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then grep -v INFO $O/pytest_gpu.log | tail -40; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], "fp32", d["fp32"]["ms_per_step"])'
