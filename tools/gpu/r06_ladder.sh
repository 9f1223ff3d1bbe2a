#!/bin/bash
# Round 6, final kernel: where C3's rate comes from, each step bit-exact -- the reference's own traversal (left-first,
# no distance culling) with every bounce traced and no primary-hit memo (flags 0x7, the tile kernel); the culled walk
# on the reference BVH (0x16); the render BVH4 wavefront walk without the dead-path skip and memo (0x6); the product.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_ladder
mkdir -p $OUT
for f in 7 22 6 0; do
  timeout -k 10 600 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-count --flags $f > $OUT/flags_$f.json 2> $OUT/flags_$f.err \
      || { echo "bench-fail $f"; tail -5 $OUT/flags_$f.err; exit 1; }
  echo "flags $f: $(python3 -c "import json;d=json.load(open('$OUT/flags_$f.json'));print(d['value'], d['ms_per_step'], d['mrays_per_s_traced'])")" | tee -a $OUT/summary.txt
done
echo done
