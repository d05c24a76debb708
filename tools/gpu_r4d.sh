#!/bin/bash
# Round 4 (d): tail-fusion diagnostics, the atomic-statistics A/B on the ResNet-50 bench, the step
# profile, Transformer beam-search kernels, the int8 VGG16 quality numbers.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
t() { local log=$1 lim=$2; shift 2; timeout -k 10 $lim $T "$@" > gpurun_out/r4d/$log 2>&1; local rc=$?
      tail -2 gpurun_out/r4d/$log; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 120 python tools/tail_diag.py > gpurun_out/r4d/tail_diag.log 2>&1 || { tail -30 gpurun_out/r4d/tail_diag.log; exit 1; }
cat gpurun_out/r4d/tail_diag.log | grep cmp
t tests_fix.log 300 tests/test_bn_prologue.py tests/test_attn_decode_native.py
for a in 0 1; do
  BIGDL_BN_ATOMICSTATS=$a timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp32-steps 0 > gpurun_out/r4d/bench_atomic$a.log 2>&1 || { tail -30 gpurun_out/r4d/bench_atomic$a.log; exit 1; }
  tail -1 gpurun_out/r4d/bench_atomic$a.log | cut -c1-200
done
bash tools/prof_resnet.sh || exit 1
cp gpurun_out/prof_rn_summary.txt gpurun_out/r4d/
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d/beam -o run -- python tools/beam_prof.py > gpurun_out/r4d/beam.log 2>&1 || { tail -30 gpurun_out/r4d/beam.log; exit 1; }
grep workload gpurun_out/r4d/beam.log
db=$(find gpurun_out/r4d/beam -name '*.db' | head -1)
python tools/rocpd_summary.py "$db" 4 60 > gpurun_out/r4d/beam_kernels.txt; rm -rf gpurun_out/r4d/beam
timeout -k 10 400 python tools/bench_configs.py --config int8 --steps 10 --warmup 3 > gpurun_out/r4d/int8.log 2>&1 || { tail -30 gpurun_out/r4d/int8.log; exit 1; }
tail -1 gpurun_out/r4d/int8.log
