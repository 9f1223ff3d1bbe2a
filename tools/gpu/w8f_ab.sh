#!/bin/bash
# Full-precision 8-wide nodes (variants/w8f: PT_WIDE8 + PT_WIDE8F) against the in-tree BVH4 kernel (GPU box,
# repo root): the GPU suite on the variant, then C3 bench lines for each library at 5 and 4 waves/SIMD.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-w8f}
mkdir -p $OUT
V=variants/w8f/libptamd.so
PT_LIB=$V timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
    > $OUT/pytest_gpu.log 2>&1
rc=$?
# (test failures are reported and the measurement goes on; a crash, abort or time limit ends the script)
[ $rc -le 1 ] || { echo "pytest-rc-$rc" > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for run in "var4 $V 4" "base5 - 5" "var5 $V 5" "base4 - 4" "var4b $V 4" "base5b - 5"; do
  set -- $run
  lib=$2; [ "$lib" = "-" ] && lib=""
  PT_LIB=$lib PT_WF_MIN_WAVES=$3 timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline \
      > $OUT/$1.json 2> $OUT/$1.err || { echo "bench-fail $1" > $OUT/done.txt; tail -5 $OUT/$1.err; exit 1; }
  echo "$1 $(python3 -c "
import json;d=json.load(open('$OUT/$1.json'));r=d['roofline'] or {}
print(d['value'], d['ms_per_step'], 'util', r.get('walk_simd_util'), 'nodes', r.get('node_fetches'), 'lds', r.get('lds_node_fetches'), 'tris', r.get('tri_tests'), 'spill', r.get('spill_entries'))")" | tee -a $OUT/summary.txt
done
echo ok > $OUT/done.txt
