#!/bin/bash
# PMC diagnostic passes (GPU box, repo root): one rocprofv3 --pmc run per counter group in PMC_GROUPS
# (groups separated by ';', counters by spaces), each over one render launch of the bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcdiag}
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-count --steps 1 --warmup 0 ${BENCH_ARGS}"
IFS=';' read -ra GS <<< "$PMC_GROUPS"
i=0
for grp in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      $B > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "pmc-fail $grp" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
