#!/bin/bash
# int8 conv epilogue VALU cut: int8 tests, short-K bench, ResNet-50 / Inception / VGG16 int8, one VALU pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_i8_native.py tests/test_int8_static.py tests/test_int8_fc.py tests/test_quantized.py > $O/tests.log 2>&1 || { grep -v INFO $O/tests.log | tail -40; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/i8_shortk_bench.py > $O/shortk.log 2>&1 || { tail -20 $O/shortk.log; exit 1; }
cat $O/shortk.log
for mdl in resnet50 inception vgg16; do
  timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model $mdl --calib 32 --steps 20 --warmup 5 > $O/int8_$mdl.log 2>&1 || { tail -30 $O/int8_$mdl.log; exit 1; }
  grep '^{' $O/int8_$mdl.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], "int8", d["ms_per_step"], "graph", d.get("int8_graph"), "bf16", d["bf16"]["ms_per_step"], "bf16c", d.get("bf16_compiled"), "cos", d["cosine_int8_vs_fp32"], "top1", d["top1_agreement"])'
done
BIGDL_I8_SHORTK=2 timeout -k 10 400 python tools/bench_configs.py --config int8 --int8-model resnet50 --calib 32 --steps 20 --warmup 5 > $O/int8_resnet50_sk2.log 2>&1 || { tail -30 $O/int8_resnet50_sk2.log; exit 1; }
grep '^{' $O/int8_resnet50_sk2.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("short-K 2:", d["config"]["model"], "int8", d["ms_per_step"], "graph", d.get("int8_graph"))'
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/pv -o run -- python3 tools/i8_shortk_bench.py 64,256,56,1 0 > $O/pv.log 2>&1 || { tail -5 $O/pv.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
m = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r6ac/pv/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_conv_i8" in r["Kernel_Name"]:
            m[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: sum(v) / len(v) for k, v in m.items()})
PY
find $O/pv -name "*.db" -delete
