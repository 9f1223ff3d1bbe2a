#!/bin/bash
# C4 whole-frame bench line (1 GPU, CPU baseline included) and the per-GPU shard rates of C3 and C4
# (bench.py --sim-shards N: one GPU's launch of an N-GPU job), on the GPU box from the repo root.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_shards}
mkdir -p $OUT
timeout -k 10 600 python3 bench.py --config C4 --steps 2 --warmup 1 > $OUT/bench_C4.json 2> $OUT/bench_C4.err \
    || { echo c4-fail > $OUT/done.txt; tail -5 $OUT/bench_C4.err; exit 1; }
echo "C4 $(python3 -c "import json;d=json.load(open('$OUT/bench_C4.json'));print(d['value'], d['ms_per_step'])")"
TAG=${TAG:-r04_shards}/shardsim_C3 bash tools/gpu/shardsim.sh || { echo c3-shard-fail > $OUT/done.txt; exit 1; }
TAG=${TAG:-r04_shards}/shardsim_C4 STEPS=2 BENCH_ARGS="--config C4" bash tools/gpu/shardsim.sh || { echo c4-shard-fail > $OUT/done.txt; exit 1; }
tail -4 $OUT/shardsim_C3/summary.txt; tail -4 $OUT/shardsim_C4/summary.txt
echo ok > $OUT/done.txt
