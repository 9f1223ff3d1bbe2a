#!/bin/bash
# Round 6, final kernel: (1) the triangle records loaded non-temporal (-DPT_TRI_AUX=2: `nt`, evict-first in L2, so the
# nodes and the shading records keep more of it) against the product, C3 alternated, with an L2 hit/miss pass each;
# (2) the whole C3 frame of the HEAD integrator against the oracle.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_exp6
mkdir -p $OUT
PT_LIB=variants/trint/libptamd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_scenes.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_trint.log 2>&1 || { echo pytest-fail; tail -20 $OUT/pytest_trint.log; exit 1; }
tail -1 $OUT/pytest_trint.log
for r in 1 2 3; do
  for v in trint base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-count > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err \
        || { echo "bench-fail $v $r"; tail -5 $OUT/${v}_$r.err; exit 1; }
    echo "$v $r $(python3 -c "import json;d=json.load(open('$OUT/${v}_$r.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
  done
done
for v in trint base; do
  lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
  PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_$v -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err \
      || { echo "pmc-fail $v"; exit 1; }
done
rm -f $OUT/fullframe_log.txt
PT_FULL_FRAME=C3H PT_FULL_FRAME_LOG=$OUT/fullframe_log.txt timeout -k 10 800 python3 -u -m pytest tests/test_gpu_fullframe_oracle.py \
    -m gpu -v --timeout 750 --timeout-method thread > $OUT/fullframe_pytest.log 2>&1 || { echo fullframe-fail; tail -30 $OUT/fullframe_pytest.log; exit 1; }
grep config $OUT/fullframe_log.txt
echo done
