#!/bin/bash
# Profile the render kernel (run on the GPU box from the repo root): kernel trace + separate PMC
# passes (each counter group in its own pass; never combined with other tracing domains).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o run -- \
    $B --steps 2 --warmup 1 > $OUT/bench_ktrace.json 2> $OUT/bench_ktrace.err || { echo ktrace-fail > $OUT/done.txt; exit 1; }
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc_$tag -o run -- \
      $B --steps 1 --warmup 0 --no-count > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { echo "pmc-fail $tag" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
