#!/bin/bash
# Build the HIP library in-tree (no-op when current), then hand the command to gpurun:
#   tools/gpurun.sh <timeout-seconds> '<command>'
set -e
cd "$(dirname "$0")/.."
(cd bigdl-1_amd && python -m bigdl.ops.build --jobs 8 >/dev/null)
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
