#!/bin/bash
# Round-2 GPU evidence: distributed path at world 1 with phase metrics, the ImageNet training CLI
# on the native loader, and a roctx marker trace of the training step.  Each GPU step has its own
# time limit; steps are chained so the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 300 env BIGDL_METRICS_JSONPATH=gpurun_out/r2/distri_metrics BIGDL_METRICS_DEVICETIMERS=1 \
  python bench.py --force-distri --steps 10 --warmup 3 > gpurun_out/r2/distri1.log 2>&1 || { tail -30 gpurun_out/r2/distri1.log; exit 1; }
tail -1 gpurun_out/r2/distri1.log
timeout -k 10 400 env PYTHONPATH=bigdl-1_amd BIGDL_METRICS_JSONPATH=gpurun_out/r2/cli_metrics python -m bigdl.models.train.imagenet \
  --synthetic 1024 -b 128 -e 1 --maxIteration 12 --depth 50 --classes 1000 --threads 8 \
  --checkpoint gpurun_out/r2/ck --summary gpurun_out/r2/sum > gpurun_out/r2/cli_imagenet.log 2>&1 || { tail -30 gpurun_out/r2/cli_imagenet.log; exit 1; }
grep -E "Iteration 12|Top1" gpurun_out/r2/cli_imagenet.log | tail -3
rm -rf gpurun_out/r2/ck
timeout -k 10 300 env BIGDL_ROCTX=1 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_mark -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/r2/prof_mark.log 2>&1 || { tail -20 gpurun_out/r2/prof_mark.log; exit 1; }
echo marker-trace done
ls -R gpurun_out/r2/prof_mark | head -20
