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
  # FULL_PMC=1: also the binding groups of tools/gpu/profile.sh and the DRAM-request pass (traffic.json's
  # `binding` and `dram_requests` blocks)
  GROUPS_=("FETCH_SIZE" "WRITE_SIZE")
  [ "$FULL_PMC" = "1" ] && GROUPS_+=("TCC_HIT_sum TCC_MISS_sum" \
      "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum" \
      "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
      "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_WR")
  for grp in "${GROUPS_[@]}"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -k 10 ${TLIM:-300} rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$c/pmc_$tag -o run -- \
        python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-count ${BENCH_ARGS} \
        > $OUT/$c/bench_$tag.json 2> $OUT/$c/bench_$tag.err || { echo "pmc-fail $c $tag" > $OUT/done.txt; exit 1; }
  done
done
echo ok > $OUT/done.txt
