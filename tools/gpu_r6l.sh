#!/bin/bash
# PTB world-1 DistriOptimizer overhead: host cProfile + kernel census, local vs distri
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
for arm in local distri; do
  f=""; [ $arm = distri ] && f="--force-distri"
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --cprofile 50 $f > $O/cp_$arm.log 2>&1 || { tail -20 $O/cp_$arm.log; exit 1; }
  grep '^{' $O/cp_$arm.log | cut -c1-200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$arm -o run -- python tools/bench_configs.py --config ptb --steps 20 --warmup 10 $f > $O/prof_$arm.log 2>&1 || { tail -20 $O/prof_$arm.log; exit 1; }
  db=$(find $O/prof_$arm -name '*.db' | head -1)
  ms=$(python -c "import json; print([json.loads(l) for l in open('$O/prof_$arm.log') if l.startswith('{\"metric')][-1]['ms_per_step']*20)")
  LAST_MS=$ms python tools/rocpd_summary.py "$db" 20 40 > $O/kern_$arm.txt; rm -rf $O/prof_$arm
  head -45 $O/kern_$arm.txt
done
# fp32 step serialised (no side-stream wgrad): true per-dispatch times of one step
BIGDL_CONV_ASYNCWGRAD=0 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/pf32 -o run -- python bench.py --dtype fp32 --steps 3 --warmup 2 --phase-steps 0 --fp32-steps 0 > $O/pf32.log 2>&1 || { tail -20 $O/pf32.log; exit 1; }
db=$(find $O/pf32 -name '*.db' | head -1)
python tools/rocpd_dispatches.py "$db" 700 > $O/fp32_dispatches.txt
ms=$(python -c "import json; print([json.loads(l) for l in open('$O/pf32.log') if l.startswith('{\"metric')][-1]['ms_per_step']*3)")
LAST_MS=$ms python tools/rocpd_summary.py "$db" 3 40 > $O/fp32_serial_summary.txt; rm -rf $O/pf32
head -12 $O/fp32_serial_summary.txt
# int8 ResNet-50 inference kernels
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/pi8 -o run -- python3 tools/bench_configs.py --config int8 --int8-model resnet50 --steps 5 --warmup 2 > $O/pi8.log 2>&1 || { tail -20 $O/pi8.log; exit 1; }
db=$(find $O/pi8 -name '*.db' | head -1)
python3 tools/rocpd_dispatches.py "$db" 1200 > $O/i8_dispatches.txt; rm -rf $O/pi8
grep metric $O/pi8.log | cut -c1-300
