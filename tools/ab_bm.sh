set -e
# A/B of wgrad k-tile depth: numerics of the pinned shape, then per-layer timings (+ block-count sweep)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BIGDL_WGRAD_BP=32 timeout -k 10 300 python -u -m pytest tests/test_native_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv" > gpurun_out/bp32_tests.log 2>&1
tail -2 gpurun_out/bp32_tests.log
BIGDL_WGRAD_BP=64 timeout -k 10 300 python -u tools/bench_conv.py --no-miopen --reps 10 --wgrad-sweep 768 --out gpurun_out/bp64.json > gpurun_out/bp64.log 2>&1
BIGDL_WGRAD_BP=32 timeout -k 10 300 python -u tools/bench_conv.py --no-miopen --reps 10 --wgrad-sweep 768,1024 --out gpurun_out/bp32.json > gpurun_out/bp32.log 2>&1
tail -1 gpurun_out/bp64.log; tail -1 gpurun_out/bp32.log
