#!/bin/bash
# Multi-process bench rehearsal on a 1-GPU box (repo root): 2 ranks sharing GPU 0 over gloo (the
# FrameLoop / shard / stats path with a host-side reduce).  RCCL itself refuses two ranks on one
# device ("Duplicate GPU detected", profiles/r02_dist_rehearsal/README.md), so its leg runs only on
# a multi-GPU node.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dist}
mkdir -p $OUT
PT_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 ${BENCH_ARGS} \
    > $OUT/gloo2.json 2> $OUT/gloo2.err || { echo "gloo fail" > $OUT/done.txt; exit 1; }
echo ok > $OUT/done.txt
