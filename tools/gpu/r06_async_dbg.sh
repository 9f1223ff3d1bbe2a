#!/bin/bash
# Round 6: does test_async_renders_on_two_streams abort on the product library when it runs without the suite's
# earlier tests (the two variant runs that aborted ran test_gpu_parity.py first)?  HIP runtime errors logged
# (AMD_LOG_LEVEL=1).  Each step stops the script on failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_async_dbg
mkdir -p $OUT
AMD_LOG_LEVEL=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k test_async_renders_on_two_streams > $OUT/alone2.log 2>&1; echo "alone rc=$?" | tee $OUT/rc.txt
tail -3 $OUT/alone2.log
grep -q "alone rc=0" $OUT/rc.txt || exit 1
# the variant subset that aborted before (test_gpu_parity.py first), on the NT-triangle variant
PT_LIB=variants/trint/libptamd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_scenes.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/trint_subset.log 2>&1 || { echo trint-subset-fail; tail -20 $OUT/trint_subset.log; exit 1; }
tail -1 $OUT/trint_subset.log
