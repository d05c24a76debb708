#!/bin/bash
# int8 conv + sum: coalesced residual epilogue; tests + ResNet-50 / Inception int8 bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_conv_i8_native.py tests/test_int8_static.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
grep -h "cosine" $O/tests.log; tail -1 $O/tests.log
for mdl in resnet50 inception; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 20 --warmup 5 > $O/int8_$mdl.log 2>&1 || { tail -30 $O/int8_$mdl.log; exit 1; }
  grep '^{' $O/int8_$mdl.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], "int8", d["ms_per_step"], "graph", d.get("int8_graph"), "bf16", d["bf16"], "bf16c", d.get("bf16_compiled"), "cos", d["cosine_int8_vs_fp32"], "top1", d["top1_agreement"])'
done
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/pi8 -o run -- python3 tools/bench_configs.py --config int8 --int8-model resnet50 --steps 5 --warmup 2 > $O/pi8.log 2>&1 || { tail -20 $O/pi8.log; exit 1; }
db=$(find $O/pi8 -name '*.db' | head -1)
python3 tools/rocpd_dispatches.py "$db" 1200 > $O/i8_dispatches.txt; rm -rf $O/pi8
