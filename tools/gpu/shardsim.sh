#!/bin/bash
# Per-GPU rate of one shard of N (bench.py --sim-shards N: shard 0 of N on this GPU; the whole-job
# rate at N GPUs is N x this), for each N in SHARDS (run on the GPU box from the repo root).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shardsim}
mkdir -p $OUT
for n in ${SHARDS:-2 4 8}; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count --sim-shards $n \
      > $OUT/s_$n.json 2> $OUT/s_$n.err || { echo "fail $n" > $OUT/done.txt; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$OUT/s_$n.json'));print(d['value'], d['ms_per_step'])")" >> $OUT/summary.txt
done
echo ok > $OUT/done.txt
