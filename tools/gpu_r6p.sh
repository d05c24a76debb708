#!/bin/bash
# fp32 BN prologue v2 (slice-1 prologue under slice-0 MFMAs): tests, A/B x3 interleaved, serial profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_bn_prologue.py tests/test_fp32_direct.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for arm in pro nopro; do
    e=""; [ $arm = nopro ] && e="BIGDL_FP32_BNPROLOGUE=0"
    env $e timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > $O/${arm}_$i.log 2>&1 || { tail -20 $O/${arm}_$i.log; exit 1; }
    echo "fp32 $arm $i $(grep metric $O/${arm}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
BIGDL_CONV_ASYNCWGRAD=0 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/pf32 -o run -- python bench.py --dtype fp32 --steps 3 --warmup 2 --phase-steps 0 --fp32-steps 0 > $O/pf32.log 2>&1 || { tail -20 $O/pf32.log; exit 1; }
db=$(find $O/pf32 -name '*.db' | head -1)
python tools/rocpd_dispatches.py "$db" 700 > $O/fp32_dispatches.txt; rm -rf $O/pf32
