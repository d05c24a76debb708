#!/bin/bash
# int8 zero-copy concat + unlinked conv->ReLU fusion: tests, Inception / ResNet-50 int8 bench, Inception trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6af
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_i8_native.py tests/test_int8_static.py tests/test_int8_fc.py tests/test_quantized.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
for mdl in inception resnet50; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 20 --warmup 5 > $O/int8_$mdl.log 2>&1 || { tail -30 $O/int8_$mdl.log; exit 1; }
  grep '^{' $O/int8_$mdl.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], "int8", d["ms_per_step"], "graph", (d.get("int8_graph") or {}).get("ms_per_step"), "bf16", d["bf16"]["ms_per_step"], "bf16c", (d.get("bf16_compiled") or {}).get("ms_per_step"), "cos", d["cosine_int8_vs_fp32"], "top1", d["top1_agreement"])'
done
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/p -o run -- python3 tools/bench_configs.py --config int8 --int8-model inception --calib 32 --steps 4 --warmup 2 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
db=$(find $O/p -name '*.db' | head -1)
python3 tools/rocpd_dispatches.py "$db" 500 > $O/d_inception.txt
rm -rf $O/p
