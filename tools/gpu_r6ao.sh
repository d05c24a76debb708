#!/bin/bash
# fp32 conv-epilogue BN statistics: repeated against fp64 (race hunt) on the stage-3/4 tail geometries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ao
mkdir -p $O
for spec in "512,2048,1,1,7" "256,1024,1,1,14" "64,256,1,1,56" "128,128,3,1,28"; do
  timeout -k 10 300 python -u tools/x3_stats_race.py $spec 150 128 > $O/race_$spec.log 2>&1 || { tail -20 $O/race_$spec.log; exit 1; }
  cat $O/race_$spec.log
done
