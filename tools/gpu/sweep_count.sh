#!/bin/bash
# counting sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweepc}
mkdir -p $OUT
i=0
for kv in ${SWEEP}; do
  i=$((i+1))
  env $(echo $kv | tr ',' ' ') timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
      > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "fail $kv" > $OUT/done.txt; exit 1; }
  echo "$kv $(python3 -c "import json;d=json.load(open('$OUT/b_$i.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['walk_simd_util'], r['walk_phase_frac'], r['shade_phases'], r['node_fetches'], r['tri_tests'])")" >> $OUT/summary.txt
done
echo ok > $OUT/done.txt
