#!/bin/bash
# Round-6 artifacts, part B2 (GPU box, repo root): one shard of 2 / 4 / 8 at C3 (the per-GPU launch of an N-GPU job) with
# FETCH/WRITE passes, the shard simulation of C3 and C4, the host-buffer (PCIe-inclusive) rates, and the plain
# `bench.py --gpus 2` launcher over gloo on this one GPU.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_final
mkdir -p $OUT
for n in 2 4 8; do
  TAG=r06_final/shard$n CONFIGS="C3" STEPS=$(( 2 * n )) BENCH_ARGS="--sim-shards $n" bash tools/gpu/configs.sh \
      || { echo "shard-fail $n" > $OUT/done_b2.txt; exit 1; }
done
echo shards ok
TAG=r06_final/shardsim_C3 bash tools/gpu/shardsim.sh || { echo shardsim-fail > $OUT/done_b2.txt; exit 1; }
TAG=r06_final/shardsim_C4 STEPS=2 BENCH_ARGS="--config C4" bash tools/gpu/shardsim.sh || { echo shardsim4-fail > $OUT/done_b2.txt; exit 1; }
echo shardsim ok
timeout -k 10 300 python3 tools/gpu/host_rate.py > $OUT/host_rate.json 2> $OUT/host_rate.err || { echo hostrate-fail > $OUT/done_b2.txt; exit 1; }
PT_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline \
    > $OUT/plain_gpus2_gloo.json 2> $OUT/plain_gpus2_gloo.err || { echo plain-fail > $OUT/done_b2.txt; exit 1; }
echo ok > $OUT/done_b2.txt
