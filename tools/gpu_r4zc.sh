#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zc
timeout -k 10 400 python -u tools/vgg_flaky.py > gpurun_out/r4zc/vgg.log 2>&1; rc=$?; grep '^{' gpurun_out/r4zc/vgg.log; [ $rc -eq 0 ] || tail -20 gpurun_out/r4zc/vgg.log
