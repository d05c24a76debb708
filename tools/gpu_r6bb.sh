#!/bin/bash
# bf16 stem weight gradient folded natively (bigdl_c4_wgrad_fold): conv tests, bench, bf16 kernel list
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6bb
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_native_kernels.py tests/test_train_parity.py tests/test_stem_input.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], "fp32", d["fp32"]["ms_per_step"])'
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b16 -o run -- python bench.py --steps 3 --warmup 3 --phase-steps 0 --fp32-steps 0 > $O/prof16.log 2>&1 || { tail -20 $O/prof16.log; exit 1; }
db=$(find gpurun_out/prof_b16 -name '*.db' | head -1)
ms=$(python -c "import json; print([json.loads(l) for l in open('$O/prof16.log') if l.startswith('{\"metric')][-1]['ms_per_step']*3)")
LAST_MS=$ms python tools/rocpd_summary.py "$db" 3 200 > $O/prof16_summary.txt; rm -rf gpurun_out/prof_b16
head -3 $O/prof16_summary.txt; echo -n "bf16 at::native kernels: "; grep -c "at::native" $O/prof16_summary.txt || true
