#!/bin/bash
# PMC counters of the product (5 waves/SIMD) against the 6-wave build (register packing, scheduler RP
# trackers, walk state parked across shading; variants/w6tp, PT_WF_MIN_WAVES=6) and the same build at 5
# waves: L2 hit rate, memory-side bytes, TD/TA busy, VALU -- why a sixth wave buys nothing.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_pmc_waves}
mkdir -p $OUT
run() {   # name -- env set by the caller
  local name=$1; shift
  mkdir -p $OUT/$name
  for grp in "TCC_HIT_sum TCC_MISS_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$name/pmc_$tag -o run -- \
        python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-count > $OUT/$name/bench_$tag.json 2> $OUT/$name/bench_$tag.err \
        || { echo "pmc-fail $name $tag" > $OUT/done.txt; exit 1; }
  done
}
run base_c3 || exit 1
PT_LIB=variants/w6tp/libptamd.so PT_WF_MIN_WAVES=6 run w6_c3 || exit 1
PT_LIB=variants/w6tp/libptamd.so run w5_c3 || exit 1
echo ok > $OUT/done.txt
