set -e
# A/B of conv tile shapes: numerics of the pinned shape, then per-layer timings of each shape
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BIGDL_CONV_BK=32 timeout -k 10 300 python -u -m pytest tests/test_native_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv or dgrad or bn_forward_from" > gpurun_out/bk32_tests.log 2>&1
tail -2 gpurun_out/bk32_tests.log
BIGDL_CONV_BK=64 timeout -k 10 300 python -u tools/bench_conv.py --no-miopen --reps 10 --out gpurun_out/bk64.json > gpurun_out/bk64.log 2>&1
BIGDL_CONV_BK=32 timeout -k 10 300 python -u tools/bench_conv.py --no-miopen --reps 10 --out gpurun_out/bk32.json > gpurun_out/bk32.log 2>&1
tail -1 gpurun_out/bk64.log; tail -1 gpurun_out/bk32.log
