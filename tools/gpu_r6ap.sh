#!/bin/bash
# after the x3 epilogue barrier fix: statistics race test, per-step BN check in training, fp32 training repeats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ap
mkdir -p $O
for spec in "256,1024,1,1,14" "512,2048,1,1,7" "1024,256,1,1,14" "128,512,1,1,28"; do
  timeout -k 10 300 python -u tools/x3_stats_race.py $spec 400 128 > $O/race_$spec.log 2>&1 || { tail -20 $O/race_$spec.log; exit 1; }
  tail -1 $O/race_$spec.log
done
timeout -k 10 600 python -u tools/convergence.py --dtype fp32 --steps 600 --batch 128 --classes 1000 --noise 2 --log-every 50 --check-bn 1 > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
grep bn_worst $O/check.log | python3 -c '
import sys, json
rows = [json.loads(l) for l in sys.stdin]
print("steps with BN invstd err > 1e-3:", sum(r["bn_worst_rel_invstd_err"] > 1e-3 for r in rows), "worst", max(r["bn_worst_rel_invstd_err"] for r in rows))'
A="--steps 700 --batch 128 --classes 1000 --noise 2 --log-every 50"
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/convergence.py --dtype fp32 $A > $O/fp32_$i.log 2>&1 || { tail -20 $O/fp32_$i.log; exit 1; }
  echo "fp32 $i $(grep '"step"' $O/fp32_$i.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["loss"]) for l in sys.stdin))') acc $(grep final $O/fp32_$i.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["heldout_acc"])')"
done
