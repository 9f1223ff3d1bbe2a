#!/bin/bash
# PMC evidence for two rejected round-4 variants (GPU box, repo root): the 6-waves/SIMD build
# (variants/w6, PT_WF_MIN_WAVES=6) against the product at C3 -- TD/TA busy, VALU, L1 lookups -- and the C2
# register-state build (variants/rs, PT_WF_REG_STATE=1) against the product -- FETCH/WRITE_SIZE -- and the
# top-nodes-from-LDS asm step (variants/topasm, profiles/r04_topasm) at C3 -- L1 lookups, TD busy.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_pmc_rej}
mkdir -p $OUT
run() {   # name env... -- bench args
  local name=$1; shift
  for grp in "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_TA_BUSY_sum" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$name/pmc_$tag -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count "$@" > $OUT/$name/bench_$tag.json 2> $OUT/$name/bench_$tag.err \
        || { echo "pmc-fail $name $tag" > $OUT/done.txt; exit 1; }
  done
}
mkdir -p $OUT/base_c3 $OUT/w6_c3 $OUT/base_c2 $OUT/rs_c2 $OUT/top_c3
run base_c3 || exit 1
PT_LIB=variants/topasm/libptamd.so run top_c3 || exit 1
PT_LIB=variants/w6/libptamd.so PT_WF_MIN_WAVES=6 run w6_c3 || exit 1
run base_c2 --config C2 || exit 1
PT_LIB=variants/rs/libptamd.so PT_WF_REG_STATE=1 run rs_c2 --config C2 || exit 1
echo ok > $OUT/done.txt
