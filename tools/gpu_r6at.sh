#!/bin/bash
# round-6 final: default bench.py x3 (bf16 headline + fp32 record), smoke, full GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6at
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  grep '^{' $O/bench_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], "fp32", d["fp32"]["ms_per_step"], d["fp32"]["value"])'
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
exit $rc
