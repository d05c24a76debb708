#!/bin/bash
# Rehearse the driver's N>1 launch on a one-GPU box: two ranks on the same card (RCCL refuses a
# duplicate GPU, so the collectives run over gloo: BIGDL_DIST_BACKEND=gloo), small per-rank batch,
# bf16 headline + fp32 record, then SyncBN; the device-side multi-rank path (bucket hooks, sharded
# update, bf16 wire, side streams) is the one RCCL runs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6bc
mkdir -p $O
BIGDL_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --fp32-steps 2 > $O/n2.log 2>&1; rc=$?
echo "rc=$rc"; grep '^{' $O/n2.log | cut -c1-900; grep -v INFO $O/n2.log | grep -i "error\|traceback" | head -20
[ $rc -eq 0 ] || exit $rc
BIGDL_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --fp32-steps 0 --syncbn > $O/n2_syncbn.log 2>&1; rc=$?
echo "syncbn rc=$rc"; grep '^{' $O/n2_syncbn.log | cut -c1-600; grep -v INFO $O/n2_syncbn.log | grep -i "error\|traceback" | head -20
grep -h "DistriOptimizer:" $O/n2.log | head -2
exit $rc
