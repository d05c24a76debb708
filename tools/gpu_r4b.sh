#!/bin/bash
# Round 4: BN/SyncBN kernel changes under test, conv PMC passes with the x8 family off / on, and the
# ResNet-50 step kernel profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_syncbn_native.py tests/test_conv_x8.py tests/test_native_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 || { tail -40 gpurun_out/r4b/tests.log; exit 1; }
tail -2 gpurun_out/r4b/tests.log
SP="256,256,3,1,14 fwd;512,512,3,1,7 fwd;1024,256,1,1,14 fwd;64,256,1,1,56 fwdstats;256,256,3,1,14 wgrad"
for v in 0 1; do
  rm -rf gpurun_out/pmc2
  BIGDL_CONV_X8=$v SPECS="$SP" bash tools/pmc_conv2.sh || exit 1
  python tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/r4b/pmc_x8_$v.txt
  rm -rf gpurun_out/pmc2
done
bash tools/prof_resnet.sh || exit 1
cp gpurun_out/prof_rn_summary.txt gpurun_out/r4b/
