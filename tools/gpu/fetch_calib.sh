#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the path tracer's access shapes (GPU box, repo root):
# the probe's kernels fetch known byte counts; one rocprofv3 --pmc pass per counter.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
B=tools/gpu/micro/fetch_calib
timeout -k 10 60 $B > $OUT/known.txt 2>&1 || { echo run-fail > $OUT/done.txt; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/p_$c -o run -- $B > $OUT/b_$c.txt 2>&1 \
      || { echo "pmc-fail $c" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
