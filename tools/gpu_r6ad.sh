#!/bin/bash
# int8 short-K tile 0 vs 2 inside the nets (3 interleaved repeats each), after the launch-geometry fix
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ad
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_i8_native.py tests/test_int8_static.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for sk in 0 2; do
    for mdl in resnet50 vgg16; do
      BIGDL_I8_SHORTK=$sk timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 20 --warmup 5 > $O/${mdl}_${sk}_$i.log 2>&1 || { tail -30 $O/${mdl}_${sk}_$i.log; exit 1; }
      echo "sk $sk rep $i $(grep '^{' $O/${mdl}_${sk}_$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], "int8", d["ms_per_step"], "graph", (d.get("int8_graph") or {}).get("ms_per_step"), "bf16c", (d.get("bf16_compiled") or {}).get("ms_per_step"))')"
    done
  done
done
