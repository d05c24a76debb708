#!/bin/bash
# fp32 BN prologue: kernel + model tests, parity, fp32 bench A/B (interleaved), serial dispatch profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_bn_prologue.py tests/test_fp32_direct.py tests/test_fp32x3.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u -m pytest -x -s -q --timeout 300 --timeout-method thread tests/test_train_parity.py -k fp32 > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
grep -A2 "fp32 ResNet-50" $O/parity.log; tail -1 $O/parity.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > $O/f32_$i.log 2>&1 || { tail -20 $O/f32_$i.log; exit 1; }
  echo "fp32 pro $i $(grep metric $O/f32_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  BIGDL_FP32_BNPROLOGUE=0 timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --fp32-steps 0 > $O/f32np_$i.log 2>&1 || { tail -20 $O/f32np_$i.log; exit 1; }
  echo "fp32 nopro $i $(grep metric $O/f32np_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
done
BIGDL_CONV_ASYNCWGRAD=0 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/pf32 -o run -- python bench.py --dtype fp32 --steps 3 --warmup 2 --phase-steps 0 --fp32-steps 0 > $O/pf32.log 2>&1 || { tail -20 $O/pf32.log; exit 1; }
db=$(find $O/pf32 -name '*.db' | head -1)
python tools/rocpd_dispatches.py "$db" 700 > $O/fp32_dispatches.txt
ms=$(python -c "import json; print([json.loads(l) for l in open('$O/pf32.log') if l.startswith('{\"metric')][-1]['ms_per_step']*3)")
LAST_MS=$ms python tools/rocpd_summary.py "$db" 3 40 > $O/fp32_serial_summary.txt; rm -rf $O/pf32
head -24 $O/fp32_serial_summary.txt
# bf16 headline (default bench) and PTB world-1 distri host profile
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench bf16", d["ms_per_step"], "fp32", d["fp32"]["ms_per_step"])'
timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --cprofile 100 --force-distri > $O/ptb_cp.log 2>&1 || { tail -20 $O/ptb_cp.log; exit 1; }
grep -A45 "function calls" $O/ptb_cp.log | head -60
