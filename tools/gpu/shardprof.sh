#!/bin/bash
# Where a small shard's time goes (GPU box, repo root): kernel trace of bench --sim-shards N (per-kernel
# durations vs the step's wall time) and one counting pass with the wall-clock dump (queue drained /
# last wave exit), for each N in SHARDS.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shardprof}
mkdir -p $OUT
for n in ${SHARDS:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$n -o run -- \
      python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-count --sim-shards $n ${BENCH_ARGS} \
      > $OUT/kt_$n.json 2> $OUT/kt_$n.err || { echo "kt fail $n" > $OUT/done.txt; exit 1; }
  PT_SECTION_DUMP=$PWD/$OUT/sections_$n.txt timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
      --sim-shards $n ${BENCH_ARGS} > $OUT/cnt_$n.json 2> $OUT/cnt_$n.err || { echo "cnt fail $n" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
