#!/bin/bash
# L1 lookups, TA / TD busy and TD_TC_STALL of the render kernel per setting (GPU box, repo root): one
# rocprofv3 --pmc pass (one launch) per entry of SETTINGS ("label:VAR=VAL,VAR2=VAL2 ...").
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-coop_pmc}
mkdir -p $OUT
for cfg in $SETTINGS; do
  label=${cfg%%:*}
  envs=${cfg#*:}
  env ${envs//,/ } timeout -s KILL 150 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv -d $OUT/pmc_$label -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline ${BENCH_ARGS} > $OUT/pmc_$label.json 2> $OUT/pmc_$label.err \
      || { echo "pmc-fail $label" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
