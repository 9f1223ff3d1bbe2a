#!/bin/bash
# Bench under a list of environment settings (run on the GPU box). SWEEP="VAR=a VAR=b ..."
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
i=0
for kv in ${SWEEP}; do
  i=$((i+1))
  env $(echo $kv | tr ',' ' ') timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count ${BENCH_ARGS} \
      > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "fail $kv" > $OUT/done.txt; exit 1; }
  echo "$kv $(python3 -c "import json;d=json.load(open('$OUT/b_$i.json'));print(d['value'], d['ms_per_step'])")" >> $OUT/summary.txt
done
echo ok > $OUT/done.txt
