#!/bin/bash
# ADVICE r05 (pt_render.hip:885): the CF_CHUNK0 invariant checked on the device (-DPT_DEBUG_CHECKS: a chunk-0 unit of a
# split slot must end at chunk_first(1) of the slot's grade, where finalize_pixels continues its running mean) over the
# GPU suite (split units, shards, C2-C5 subsets) and full C3 / shard frames; then three fresh C3 bench runs of the product.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_debugchecks
mkdir -p $OUT
PT_LIB=variants/debugchecks/libptamd.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for n in 1 2 4 8; do
  PT_LIB=variants/debugchecks/libptamd.so timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count --sim-shards $n \
      > $OUT/shard_$n.json 2> $OUT/shard_$n.err || { echo "shard-fail $n"; tail -5 $OUT/shard_$n.err; exit 1; }
  echo "debug build, shard 0 of $n: $(python3 -c "import json;d=json.load(open('$OUT/shard_$n.json'));print(d['value'], d['image_finite'])")"
done
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { echo bench-fail; exit 1; }
  echo "product bench $r: $(python3 -c "import json;d=json.load(open('$OUT/bench_$r.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['bound'])")"
done
echo done
