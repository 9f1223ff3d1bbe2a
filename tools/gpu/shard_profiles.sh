#!/bin/bash
# Kernel trace + FETCH_SIZE / WRITE_SIZE passes of one shard of N (bench --sim-shards N: the per-GPU
# launch of an N-GPU job) for each N in SHARDS, so that the N-GPU bench lines carry a measured roofline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shardprof}
mkdir -p $OUT
for n in ${SHARDS:-2 4 8}; do
  TAG=${TAG:-shardprof}/s$n CONFIGS="C3" STEPS=$(( 2 * n )) BENCH_ARGS="--sim-shards $n" bash tools/gpu/configs.sh \
      || { echo "fail $n" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
