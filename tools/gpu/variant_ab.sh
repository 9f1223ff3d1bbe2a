#!/bin/bash
# Experiment-variant A/B (GPU box, repo root): the GPU suite on the variant library (VARIANT, a
# variants/<name>/libptamd.so built by tools/build_variants.sh; NOTEST=1 skips it), then the C3 bench with
# its counting pass on the variant and on the in-tree library, alternated ROUNDS times (default 2).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-variant}
mkdir -p $OUT
V=variants/${VARIANT:?}/libptamd.so
if [ -z "$NOTEST" ]; then
  PT_LIB=$V timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
      > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for r in $(seq ${ROUNDS:-2}); do
  for lib in "$V" ""; do
    tag=$([ -n "$lib" ] && echo var || echo base)_$r
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/$tag.json 2> $OUT/$tag.err \
        || { echo "bench-fail $tag" > $OUT/done.txt; tail -5 $OUT/$tag.err; exit 1; }
    echo "$tag $(python3 -c "
import json;d=json.load(open('$OUT/$tag.json'));r=d['roofline'] or {}
print(d['value'], d['ms_per_step'], 'util', r.get('walk_simd_util'), 'walkfrac', r.get('walk_phase_frac'), 'nodes', r.get('node_fetches'), 'lds', r.get('lds_node_fetches'), 'tris', r.get('tri_tests'), 'spill', r.get('spill_entries'))")" | tee -a $OUT/summary.txt
  done
done
echo ok > $OUT/done.txt
