#!/bin/bash
# Experiment run (GPU box, repo root): GPU parity tests under $TEST_ENV, then a bench per
# setting in SWEEP ("VAR=a,VAR2=b VAR=c ..."; "-" = defaults), with the counting pass when COUNT=1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-exp}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  env $TEST_ENV timeout -k 10 600 python3 -m pytest tests -x -q -m gpu $TESTS > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed" > $OUT/done.txt; exit 1; }
fi
i=0
for kv in ${SWEEP:--}; do
  i=$((i+1))
  envs=""; [ "$kv" != "-" ] && envs=$(echo $kv | tr ',' ' ')
  cnt="--no-count"; [ "$COUNT" = "1" ] && cnt=""
  env $envs PT_SECTION_DUMP=$PWD/$OUT/sections_$i.txt timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $cnt ${BENCH_ARGS} \
      > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "bench failed: $kv" > $OUT/done.txt; exit 1; }
  echo "$kv $(python3 -c "
import json;d=json.load(open('$OUT/b_$i.json'));r=d['roofline'] or {};print(d['value'], d['ms_per_step'], r.get('walk_simd_util'), r.get('walk_phase_frac'), r.get('shade_phases'), r.get('node_fetches'), r.get('tri_tests'))")" >> $OUT/summary.txt
done
echo ok > $OUT/done.txt
