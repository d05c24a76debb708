#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_step_bytes.sh --fp32-steps 0 || exit 1
