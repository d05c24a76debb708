#!/bin/bash
# conv shape table with a tuned vendor baseline (MIOpen NORMAL find + cudnn.benchmark), bs 256 bf16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
VENDOR_CONV=1 MIOPEN_FIND_MODE=NORMAL VENDOR_BENCH=1 timeout -k 10 1000 python -u tools/pw_bench.py > $O/pw_tuned.jsonl 2> $O/pw_tuned.err || { tail -20 $O/pw_tuned.err; tail -5 $O/pw_tuned.jsonl; exit 1; }
tail -3 $O/pw_tuned.jsonl
