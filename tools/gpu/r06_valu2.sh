#!/bin/bash
# The VALU issue-cost probe with launches long enough to amortise dispatch (kIters 8192).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_valu
mkdir -p $OUT
timeout -k 10 300 tools/gpu/micro/valu_cost > $OUT/valu_cost3.txt 2>&1 || { echo probe-fail; cat $OUT/valu_cost3.txt; exit 1; }
cat $OUT/valu_cost3.txt
