#!/bin/bash
# BN-statistics check in bf16 training; a longer fp32 native run (2000 steps) next to torch fp32 (700)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ar
mkdir -p $O
timeout -k 10 400 python -u tools/convergence.py --dtype bf16 --steps 400 --batch 128 --classes 1000 --noise 2 --log-every 50 --check-bn 1 > $O/check_bf16.log 2>&1 || { tail -20 $O/check_bf16.log; exit 1; }
grep bn_worst $O/check_bf16.log | python3 -c '
import sys, json
rows = [json.loads(l) for l in sys.stdin]
print("bf16: steps with BN invstd err > 1e-2:", sum(r["bn_worst_rel_invstd_err"] > 1e-2 for r in rows), "worst", max(r["bn_worst_rel_invstd_err"] for r in rows))'
timeout -k 10 600 python -u tools/convergence.py --dtype fp32 --steps 2000 --batch 128 --classes 1000 --noise 2 --log-every 100 > $O/fp32_long.log 2>&1 || { tail -20 $O/fp32_long.log; exit 1; }
grep '"step"' $O/fp32_long.log | python3 -c 'import sys,json; print("fp32 2000:", " ".join(str(json.loads(l)["loss"]) for l in sys.stdin))'
grep final $O/fp32_long.log
