#!/bin/bash
# Iteration check (GPU box, repo root): GPU parity tests, then the default bench line.
# TESTS="..." narrows the tests (pytest -k); NOTEST=1 skips them.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
      > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err \
    || { echo bench-fail > $OUT/done.txt; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'] or {}
print('value', d['value'], 'ms', d['ms_per_step'], 'util', r.get('walk_simd_util'), 'walkfrac', r.get('walk_phase_frac'), 'passes', r.get('shade_phases'), 'nodes', r.get('node_fetches'), 'lds', r.get('lds_node_fetches'), 'tris', r.get('tri_tests'))"
echo ok > $OUT/done.txt
