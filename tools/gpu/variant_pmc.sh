#!/bin/bash
# TD / TA busy, VALU instructions and cycles of the render kernel for the variant (VARIANT) and the in-tree
# library: one rocprofv3 --pmc pass each (one launch), then the variant's bench under each setting in SWEEP.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-vpmc}
mkdir -p $OUT
V=variants/${VARIANT:?}/libptamd.so
for lib in "$V" ""; do
  tag=$([ -n "$lib" ] && echo var || echo base)
  PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc ${PMC:-TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD} \
      --kernel-trace --output-format csv -d $OUT/pmc_$tag -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_$tag.json 2> $OUT/pmc_$tag.err \
      || { echo "pmc-fail $tag" > $OUT/done.txt; exit 1; }
done
i=0
for kv in ${SWEEP:--}; do
  i=$((i+1))
  envs=""; [ "$kv" != "-" ] && envs=$(echo $kv | tr ',' ' ')
  env $envs PT_LIB=$V timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count > $OUT/s_$i.json 2> $OUT/s_$i.err \
      || { echo "bench-fail $kv" > $OUT/done.txt; exit 1; }
  echo "$kv $(python3 -c "import json;d=json.load(open('$OUT/s_$i.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
done
echo ok > $OUT/done.txt
