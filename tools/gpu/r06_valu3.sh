#!/bin/bash
# The walk step's VALU stream replayed alone (tools/gpu/micro/walk_replay), then the issue-cost probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_valu
mkdir -p $OUT
timeout -k 10 120 tools/gpu/micro/walk_replay > $OUT/walk_replay2.txt 2>&1 || { echo replay-fail; cat $OUT/walk_replay2.txt; exit 1; }
cat $OUT/walk_replay2.txt
