#!/bin/bash
# Round artifacts, part B (GPU box, repo root): C2 / C5 bench lines with kernel trace and FETCH/WRITE passes,
# the same for integrator 1 at C3, the shard simulation, and the host-buffer (PCIe-inclusive) rates.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
TAG=${TAG:-final}/configs CONFIGS="C2 C5" bash tools/gpu/configs.sh || { echo configs-fail > $OUT/done_b.txt; exit 1; }
echo configs ok
TAG=${TAG:-final}/head CONFIGS="C3" BENCH_ARGS="--integrator 1" bash tools/gpu/configs.sh || { echo head-fail > $OUT/done_b.txt; exit 1; }
echo head ok
TAG=${TAG:-final}/shardsim bash tools/gpu/shardsim.sh || { echo shardsim-fail > $OUT/done_b.txt; exit 1; }
echo shardsim ok
timeout -k 10 300 python3 tools/gpu/host_rate.py > $OUT/host_rate.json 2> $OUT/host_rate.err || { echo hostrate-fail > $OUT/done_b.txt; exit 1; }
echo ok > $OUT/done_b.txt
