#!/bin/bash
# Round 6, miss-latency diagnostic: 64-B triangle records (-DPT_TRI64: +33% footprint of the triangle arrays, the same
# instructions) against the product, C3 alternated, and one L2 hit/miss pass each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_exp5c
mkdir -p $OUT
PT_LIB=variants/tri64/libptamd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_random_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_tri64.log 2>&1 || { echo pytest-fail; tail -20 $OUT/pytest_tri64.log; exit 1; }
tail -1 $OUT/pytest_tri64.log
for r in 1 2 3; do
  for v in tri64 base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err \
        || { echo "bench-fail $v $r"; tail -5 $OUT/${v}_$r.err; exit 1; }
    echo "$v $r $(python3 -c "import json;d=json.load(open('$OUT/${v}_$r.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['node_fetches'], r['tri_tests'])")" | tee -a $OUT/summary.txt
  done
done
for pmc in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  for v in tri64 base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $OUT/pmc_${v}_$tag -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_${v}_$tag.json 2> $OUT/pmc_${v}_$tag.err \
        || { echo "pmc-fail $v $tag"; exit 1; }
  done
done
echo done
