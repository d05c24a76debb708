#!/bin/bash
# Inception-v1 eager inference: round-3 tree vs HEAD — kernel time per step and host profile
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6r
mkdir -p $O
for tree in r3 head; do
  d=.; [ $tree = r3 ] && d=ab_r3
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p_$tree -o run -- python tools/bench_configs.py --config inception --steps 20 --warmup 5 > $O/prof_$tree.log 2>&1) || { tail -20 $O/prof_$tree.log; exit 1; }
  db=$(find $O/p_$tree -name '*.db' | head -1)
  ms=$(python -c "import json; print([json.loads(l) for l in open('$O/prof_$tree.log') if l.startswith('{')][-1]['ms_per_step']*20)")
  LAST_MS=$ms python tools/rocpd_summary.py "$db" 20 30 > $O/kern_$tree.txt; rm -rf $O/p_$tree
  head -22 $O/kern_$tree.txt
  (cd $d && timeout -k 10 300 python tools/bench_configs.py --config inception --steps 20 --warmup 5 --cprofile 20 > $O/cp_$tree.log 2>&1) || { tail -20 $O/cp_$tree.log; exit 1; }
  grep -A30 "function calls" $O/cp_$tree.log | head -36
done
