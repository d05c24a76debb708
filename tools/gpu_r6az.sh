#!/bin/bash
# fp32/bf16 step without torch kernels: native arena clear (bigdl_fill32) and float-target cross
# entropy; kernel tests, the bench line, then the fp32 step's full kernel list (at::native count)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6az
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_native_kernels.py tests/test_no_fallback.py tests/test_train_parity.py tests/test_fp32_direct.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], "fp32", d["fp32"]["ms_per_step"])'
TOP=200 bash tools/prof_fp32.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -3 gpurun_out/prof_f32_summary.txt; echo -n "at::native kernels: "; grep -c "at::native" gpurun_out/prof_f32_summary.txt || true
DTYPE=fp32 B=256 DEVICE_ONLY=1 DISPATCH=1 timeout -k 10 300 python tools/torch_prof_step.py > $O/tps32.log 2>&1 || { tail -20 $O/tps32.log; exit 1; }
sed -n '/dispatch sites/,$p' $O/tps32.log
DTYPE=bf16 B=256 DEVICE_ONLY=1 DISPATCH=1 timeout -k 10 300 python tools/torch_prof_step.py > $O/tps16.log 2>&1 || { tail -20 $O/tps16.log; exit 1; }
sed -n '/dispatch sites/,$p' $O/tps16.log
