#!/bin/bash
# fp32 native: per-step check of every BN's batch statistics against fp64 statistics of its input
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6an
mkdir -p $O
timeout -k 10 600 python -u tools/convergence.py --dtype fp32 --steps 600 --batch 128 --classes 1000 --noise 2 --log-every 50 --check-bn 1 > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
grep -c bn_worst $O/check.log; grep bn_worst $O/check.log | python3 -c '
import sys, json
rows = [json.loads(l) for l in sys.stdin]
big = [r for r in rows if r["bn_worst_rel_invstd_err"] > 1e-3]
print("steps with invstd err > 1e-3:", len(big))
for r in sorted(rows, key=lambda r: -r["bn_worst_rel_invstd_err"])[:12]: print(r)'
grep '"loss"' $O/check.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["loss"]) for l in sys.stdin))'
