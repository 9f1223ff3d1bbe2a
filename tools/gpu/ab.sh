#!/bin/bash
# Same-box A/B of bench configurations (GPU box, repo root).
#   CONFIGS="label:VAR=VAL,VAR2=VAL2 label2: ..."  (an empty env = the in-tree library, defaults)
#   TEST=1: smoke + the GPU suite first (in-tree library; TESTENV="VAR=VAL,..." for the suite); ROUNDS (default 2);
#   BENCH_ARGS: extra bench.py arguments (e.g. --config C2); STEPS (default 4).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ -n "$TEST" ]; then
  timeout -k 10 300 python3 __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke-fail > $OUT/done.txt; tail -20 $OUT/smoke.log; exit 1; }
  echo "smoke ok"
  timeout -k 10 900 env ${TESTENV//,/ } python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
      > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail > $OUT/done.txt; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for r in $(seq ${ROUNDS:-2}); do
  for cfg in $CONFIGS; do
    label=${cfg%%:*}
    envs=${cfg#*:}
    tag=${label}_$r
    timeout -k 10 400 env ${envs//,/ } python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline ${NOCOUNT:---no-count} ${BENCH_ARGS} \
        > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench-fail $tag" > $OUT/done.txt; tail -5 $OUT/$tag.err; exit 1; }
    echo "$tag $(python3 -c "
import json;d=json.load(open('$OUT/$tag.json'));r=d.get('roofline') or {}
print(d['value'], d['ms_per_step'], 'kms', r.get('kernel_ms'), 'util', r.get('walk_simd_util'), 'nodes', r.get('node_fetches'), 'tris', r.get('tri_tests'))")" | tee -a $OUT/summary.txt
  done
done
echo ok > $OUT/done.txt
