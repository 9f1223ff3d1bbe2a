#!/bin/bash
# Round-6 artifacts, part B (GPU box, repo root): C2 / C4 / C5 bench lines with kernel trace and FETCH/WRITE
# passes, the same for integrator 1 at C3 and for one shard of 2 / 4 / 8 at C3 (the per-GPU launch of an
# N-GPU job), the shard simulation of C3 and C4, and the host-buffer (PCIe-inclusive) rates.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_final}
mkdir -p $OUT
TAG=${TAG:-r06_final}/configs FULL_PMC=1 CONFIGS="${CFGS:-C2 C4 C5}" TLIM=400 bash tools/gpu/configs.sh || { echo configs-fail > $OUT/done_b.txt; exit 1; }
echo configs ok
TAG=${TAG:-r06_final}/head FULL_PMC=1 CONFIGS="C3" BENCH_ARGS="--integrator 1" bash tools/gpu/configs.sh || { echo head-fail > $OUT/done_b.txt; exit 1; }
echo head ok
for n in 2 4 8; do
  TAG=${TAG:-r06_final}/shard$n CONFIGS="C3" STEPS=$(( 2 * n )) BENCH_ARGS="--sim-shards $n" bash tools/gpu/configs.sh \
      || { echo "shard-fail $n" > $OUT/done_b.txt; exit 1; }
done
echo shards ok
TAG=${TAG:-r06_final}/shardsim_C3 bash tools/gpu/shardsim.sh || { echo shardsim-fail > $OUT/done_b.txt; exit 1; }
TAG=${TAG:-r06_final}/shardsim_C4 STEPS=2 BENCH_ARGS="--config C4" bash tools/gpu/shardsim.sh || { echo shardsim4-fail > $OUT/done_b.txt; exit 1; }
echo shardsim ok
timeout -k 10 300 python3 tools/gpu/host_rate.py > $OUT/host_rate.json 2> $OUT/host_rate.err || { echo hostrate-fail > $OUT/done_b.txt; exit 1; }
echo ok > $OUT/done_b.txt
