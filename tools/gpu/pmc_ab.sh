#!/bin/bash
# One PMC group over one render launch for each library in LIBS (GPU box, repo root):
# A/B of dynamic instruction counts. PMC="counters ..." (one pass, within the block limits).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcab}
mkdir -p $OUT
i=0
for lib in ${LIBS}; do
  i=$((i+1))
  env PT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu-baseline --no-count --steps 1 --warmup 0 ${BENCH_ARGS} > $OUT/b_$i.json 2> $OUT/b_$i.err \
      || { echo "pmc-fail $lib" > $OUT/done.txt; exit 1; }
  python3 - "$OUT/p$i/run_counter_collection.csv" "$lib" >> $OUT/summary.txt <<'PY'
import csv, collections, sys
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "render_unidir" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], " ".join("%s=%.4g" % kv for kv in sorted(agg.items())))
PY
done
echo ok > $OUT/done.txt
