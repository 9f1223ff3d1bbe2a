#!/bin/bash
# A variant (VARIANT) against the in-tree library at 5 and 4 waves/SIMD (GPU box, repo root): the GPU suite on
# the variant (a failure is reported, a crash ends the script), then alternated C3 bench lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-waves}
mkdir -p $OUT
V=variants/${VARIANT:?}/libptamd.so
if [ -z "$NOTEST" ]; then
  PT_LIB=$V timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  [ $rc -le 1 ] || { echo "pytest-rc-$rc" > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
RUNS=${RUNS:-var5:V:5 base5:-:5 var4:V:4 var5b:V:5 base5b:-:5 var4b:V:4}
for run in $RUNS; do
  IFS=: read name lib wv <<< "$run"
  [ "$lib" = "V" ] && lib=$V || lib=""
  PT_LIB=$lib PT_WF_MIN_WAVES=$wv timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
      > $OUT/$name.json 2> $OUT/$name.err || { echo "bench-fail $name" > $OUT/done.txt; tail -5 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "
import json;d=json.load(open('$OUT/$name.json'));r=d['roofline'] or {}
print(d['value'], d['ms_per_step'], 'util', r.get('walk_simd_util'), 'nodes', r.get('node_fetches'), 'spill', r.get('spill_entries'))")" | tee -a $OUT/summary.txt
done
echo ok > $OUT/done.txt
