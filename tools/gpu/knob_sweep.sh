#!/bin/bash
# Knob sweep of the default bench (frames on two streams) for the full frame and shard 0 of 8 (SHARDS):
# each setting in SWEEP ("VAR=a,VAR2=b ..."; "-" = defaults), no counting pass.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-knobs}
mkdir -p $OUT
for n in ${SHARDS:-1 8}; do
  steps=$(( ${STEPS:-4} * (n > 1 ? n / 2 : 1) ))
  i=0
  for kv in ${SWEEP:--}; do
    i=$((i+1))
    envs=""; [ "$kv" != "-" ] && envs=$(echo $kv | tr ',' ' ')
    env $envs timeout -k 10 300 python3 bench.py --steps $steps --warmup 2 --no-cpu-baseline --no-count --sim-shards $n ${BENCH_ARGS} \
        > $OUT/s${n}_$i.json 2> $OUT/s${n}_$i.err || { echo "fail $n $kv" > $OUT/done.txt; exit 1; }
    echo "shards $n $kv $(python3 -c "import json;d=json.load(open('$OUT/s${n}_$i.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
  done
done
echo ok > $OUT/done.txt
