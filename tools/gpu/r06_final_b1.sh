#!/bin/bash
# Round-6 artifacts, part B1 (GPU box, repo root): C2 / C4 / C5 bench lines with kernel trace and the full PMC passes,
# the same for integrator 1 at C3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_final
mkdir -p $OUT
TAG=r06_final/configs FULL_PMC=1 CONFIGS="${CFGS:-C2 C4 C5}" TLIM=400 bash tools/gpu/configs.sh || { echo configs-fail > $OUT/done_b1.txt; exit 1; }
echo configs ok
TAG=r06_final/head FULL_PMC=1 CONFIGS="C3" BENCH_ARGS="--integrator 1" bash tools/gpu/configs.sh || { echo head-fail > $OUT/done_b1.txt; exit 1; }
echo head ok
echo ok > $OUT/done_b1.txt
