#!/bin/bash
# Round 6, final kernel, L2 residency: the shading records loaded and stored non-temporal (-DPT_REC_AUX=2: evict-first,
# so the walk's nodes and triangles keep more of each XCD's L2) against the product -- parity subset, C3 alternated, an
# L2 hit/miss pass each; then the 64-B triangle-record diagnostic again (its earlier abort was the runtime order).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_exp7
mkdir -p $OUT
PT_LIB=variants/recnt/libptamd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_scenes.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_recnt.log 2>&1 || { echo pytest-fail; tail -20 $OUT/pytest_recnt.log; exit 1; }
tail -1 $OUT/pytest_recnt.log
for r in 1 2 3; do
  for v in recnt base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-count > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err \
        || { echo "bench-fail $v $r"; tail -5 $OUT/${v}_$r.err; exit 1; }
    echo "$v $r $(python3 -c "import json;d=json.load(open('$OUT/${v}_$r.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
  done
done
for v in recnt base; do
  lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
  PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_$v -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err \
      || { echo "pmc-fail $v"; exit 1; }
done
bash tools/gpu/r06_exp5.sh || exit 1
echo done
