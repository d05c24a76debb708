set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_conv.py --no-miopen --reps 10 --out gpurun_out/bcdef.json > gpurun_out/bcdef.log 2>&1
tail -1 gpurun_out/bcdef.log
timeout -k 10 300 python -u tools/bench_conv.py --no-miopen --reps 10 --out gpurun_out/bcdef2.json > gpurun_out/bcdef2.log 2>&1
tail -1 gpurun_out/bcdef2.log
