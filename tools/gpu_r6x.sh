#!/bin/bash
# PTB world-1: LocalOptimizer vs forced DistriOptimizer — host profile and GPU busy fraction
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6x
mkdir -p $O
for arm in local distri; do
  f=""; [ $arm = distri ] && f="--force-distri"
  timeout -k 10 200 python tools/bench_configs.py --config ptb --steps 50 --warmup 10 --cprofile 100 $f > $O/cp_$arm.log 2>&1 || { tail -20 $O/cp_$arm.log; exit 1; }
  grep '^{' $O/cp_$arm.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["driver"], d["ms_per_step"])'
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p_$arm -o run -- python3 tools/bench_configs.py --config ptb --steps 30 --warmup 10 $f > $O/p_$arm.log 2>&1 || { tail -20 $O/p_$arm.log; exit 1; }
  db=$(find $O/p_$arm -name '*.db' | head -1)
  ms=$(grep '^{' $O/p_$arm.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')
  w=$(python -c "print($ms*20)")
  echo "$arm traced step $ms ms: $(python3 tools/rocpd_busy.py $db $w 20)"
  LAST_MS=$w python3 tools/rocpd_summary.py $db 20 30 > $O/k_$arm.txt
  rm -rf $O/p_$arm
done
