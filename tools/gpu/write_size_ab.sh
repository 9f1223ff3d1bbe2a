#!/bin/bash
# WRITE_SIZE of one C3 render launch for the variant (VARIANT) and the in-tree library (GPU box, repo root):
# one rocprofv3 --pmc pass each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wsize}
mkdir -p $OUT
V=variants/${VARIANT:?}/libptamd.so
for lib in "$V" ""; do
  tag=$([ -n "$lib" ] && echo var || echo base)
  PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_$tag -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_$tag.json 2> $OUT/pmc_$tag.err \
      || { echo "pmc-fail $tag" > $OUT/done.txt; exit 1; }
done
echo ok > $OUT/done.txt
