#!/bin/bash
# HBM (DRAM) request counters against the memory-side ones (GPU box, repo root).
# 1. tools/gpu/micro/fetch_calib on known shapes: streamed past the Infinity Cache (every line from HBM),
#    a 32 MiB table gathered again after a warm launch (Infinity-Cache resident), a 2 MiB table (L2
#    resident), 32 MiB of cells read+written twice.
# 2. one render launch of the bench config (BENCH_ARGS) with the same counter groups.
# One rocprofv3 --pmc pass per group (<= 4 TCC counters each), --kernel-trace only beside it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dram}
mkdir -p $OUT
B=tools/gpu/micro/fetch_calib
GROUPS_=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum"
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum"
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
timeout -k 10 60 $B > $OUT/known.txt 2>&1 || { echo calib-run-fail > $OUT/done.txt; exit 1; }
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/calib_p$i -o run -- $B \
      > $OUT/calib_b$i.txt 2>&1 || { echo "calib-pmc-fail $grp" > $OUT/done.txt; exit 1; }
done
echo calib-ok > $OUT/done.txt
[ -n "$NO_BENCH" ] && exit 0
BB="python3 bench.py --no-cpu-baseline --no-count --steps 1 --warmup 0 ${BENCH_ARGS}"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/bench_p$i -o run -- \
      $BB > $OUT/bench_b$i.json 2> $OUT/bench_b$i.err || { echo "bench-pmc-fail $grp" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
