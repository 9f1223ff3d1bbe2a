#!/bin/bash
# Bench lines of the BASELINE configs beyond the headline C3 (GPU box, repo root): for each config in
# CONFIGS (default "C2 C5"), the bench line with its counting pass, a kernel trace (--stats) of the
# same command and the FETCH_SIZE / WRITE_SIZE passes (each its own rocprofv3 --pmc run, one launch).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-configs}
mkdir -p $OUT
for c in ${CONFIGS:-C2 C5}; do
  mkdir -p $OUT/$c
  B="python3 bench.py --config $c --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS}"
  timeout -k 10 ${TLIM:-300} $B > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench-fail $c" > $OUT/done.txt; exit 1; }
  [ "$PROF" = "0" ] && continue
  timeout -k 10 ${TLIM:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c/ktrace -o run -- \
      $B --no-cpu-baseline --no-count > $OUT/$c/bench_ktrace.json 2> $OUT/$c/bench_ktrace.err || { echo "ktrace-fail $c" > $OUT/done.txt; exit 1; }
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 ${TLIM:-300} rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$c/pmc_$grp -o run -- \
        python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-count ${BENCH_ARGS} \
        > $OUT/$c/bench_$grp.json 2> $OUT/$c/bench_$grp.err || { echo "pmc-fail $c $grp" > $OUT/done.txt; exit 1; }
  done
done
echo ok > $OUT/done.txt
