set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bnb
timeout -k 10 200 python tools/bench_bn32.py > gpurun_out/bnb/bn32.log 2>&1 || { tail -20 gpurun_out/bnb/bn32.log; exit 1; }
cat gpurun_out/bnb/bn32.log | grep '^{'
timeout -k 10 200 python tools/stream_roofline.py > gpurun_out/bnb/roof.log 2>&1 || { tail -20 gpurun_out/bnb/roof.log; exit 1; }
grep '^{' gpurun_out/bnb/roof.log | tail -40
