#!/bin/bash
# host cost of the BN calls per ResNet-50 step: syncbn (one-rank local kernels) vs syncmr (multi-rank
# kernels at world 1), whole-run cProfile of bench.py; int8 ResNet-50 A/B of the short-K tile and FC head
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ab
mkdir -p $O
for cfg in syncbn syncmr; do
  e=""; [ $cfg = syncmr ] && e="BIGDL_BN_SYNCONERANKLOCAL=0"
  env $e timeout -k 10 300 python -m cProfile -o $O/$cfg.prof bench.py --steps 20 --warmup 5 --fp32-steps 0 --force-distri --syncbn > $O/cp_$cfg.log 2>&1 || { tail -20 $O/cp_$cfg.log; exit 1; }
  grep metric $O/cp_$cfg.log | tail -1 | cut -c1-200
  python -c "
import pstats; s = pstats.Stats('$O/$cfg.prof'); s.sort_stats('tottime').print_stats(30)
s.sort_stats('cumulative').print_stats('normalization|native_ops|containers', 40)" > $O/cp_$cfg.txt
done
for v in 0 2; do
  for fc in 0 1; do
    BIGDL_I8_SHORTK=$v timeout -k 10 300 python tools/bench_configs.py --config int8 --int8-model resnet50 --calib 32 --steps 20 --warmup 5 --int8-fc $fc > $O/i8_${v}_$fc.log 2>&1 || { tail -30 $O/i8_${v}_$fc.log; exit 1; }
    echo "shortk $v fc $fc $(grep '^{' $O/i8_${v}_$fc.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("int8_graph"), d["cosine_int8_vs_fp32"])')"
  done
done
