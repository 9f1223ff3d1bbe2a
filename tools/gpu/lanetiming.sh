#!/bin/bash
# Lane-end timing of the real (non-counting) render kernel (GPU box, repo root): bench with
# PT_LANE_TIMING for each shard count in SHARDS and each env setting in SWEEP ("-" = defaults).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lanetiming}
mkdir -p $OUT
i=0
for kv in ${SWEEP:--}; do
  i=$((i+1))
  envs=""; [ "$kv" != "-" ] && envs=$(echo $kv | tr ',' ' ')
  for n in ${SHARDS:-1 8}; do
    env $envs PT_LANE_TIMING=$PWD/$OUT/timing_${i}_$n.txt timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 \
        --no-cpu-baseline --no-count --sim-shards $n ${BENCH_ARGS} > $OUT/b_${i}_$n.json 2> $OUT/b_${i}_$n.err \
        || { echo "fail $kv $n" > $OUT/done.txt; exit 1; }
    echo "$kv $n $(python3 -c "import json;d=json.load(open('$OUT/b_${i}_$n.json'));print(d['value'], d['ms_per_step'])") $(tail -1 $OUT/timing_${i}_$n.txt)" >> $OUT/summary.txt
  done
done
echo ok > $OUT/done.txt
