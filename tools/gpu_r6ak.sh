#!/bin/bash
# int8 pixel-pair path for 64-channel 1x1 convs: tests, ResNet-50 int8 (3 repeats), per-launch trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ak
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_i8_native.py tests/test_int8_static.py tests/test_int8_fc.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model resnet50 --calib 32 --steps 20 --warmup 5 > $O/int8_$i.log 2>&1 || { tail -30 $O/int8_$i.log; exit 1; }
  grep '^{' $O/int8_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], "int8", d["ms_per_step"], "graph", (d.get("int8_graph") or {}).get("ms_per_step"), "bf16c", (d.get("bf16_compiled") or {}).get("ms_per_step"), "cos", d["cosine_int8_vs_fp32"], "top1", d["top1_agreement"])'
done
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/p -o run -- python3 tools/bench_configs.py --config int8 --int8-model resnet50 --calib 32 --steps 4 --warmup 2 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
db=$(find $O/p -name '*.db' | head -1)
python3 tools/rocpd_dispatches.py "$db" 400 > $O/d_resnet50.txt
rm -rf $O/p
