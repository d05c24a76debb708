#!/bin/bash
# Round 4: validation of the changed kernels, conv PMC passes with the x8 family off / on, the
# ResNet-50 step profile + bench (training compile phase on), then the new kernels' tests and the
# int8 VGG16 bench.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_syncbn_native.py tests/test_conv_x8.py tests/test_native_kernels.py tests/test_compiled.py > gpurun_out/r4b/tests.log 2>&1 || { tail -40 gpurun_out/r4b/tests.log; exit 1; }
tail -2 gpurun_out/r4b/tests.log
SP="256,256,3,1,14 fwd;512,512,3,1,7 fwd;1024,256,1,1,14 fwd;64,256,1,1,56 fwdstats;256,256,3,1,14 wgrad"
for v in 0 1; do
  rm -rf gpurun_out/pmc2
  BIGDL_CONV_X8=$v SPECS="$SP" bash tools/pmc_conv2.sh || exit 1
  python tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/r4b/pmc_x8_$v.txt
  rm -rf gpurun_out/pmc2
done
echo pmc ok
bash tools/prof_resnet.sh || exit 1
cp gpurun_out/prof_rn_summary.txt gpurun_out/r4b/
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4b/bench.log 2>&1 || { tail -30 gpurun_out/r4b/bench.log; exit 1; }
tail -1 gpurun_out/r4b/bench.log
timeout -k 10 300 $T tests/test_attn_decode_native.py tests/test_attention_native.py tests/test_attention_module_native.py > gpurun_out/r4b/tests_attn.log 2>&1 || { tail -40 gpurun_out/r4b/tests_attn.log; exit 1; }
tail -2 gpurun_out/r4b/tests_attn.log
timeout -k 10 300 $T tests/test_conv_i8_native.py tests/test_quantized.py > gpurun_out/r4b/tests_i8.log 2>&1 || { tail -40 gpurun_out/r4b/tests_i8.log; exit 1; }
tail -2 gpurun_out/r4b/tests_i8.log
timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r4b/int8.log 2>&1 || { tail -30 gpurun_out/r4b/int8.log; exit 1; }
tail -1 gpurun_out/r4b/int8.log
