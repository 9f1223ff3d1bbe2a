#!/bin/bash
# Round artifacts (run on the GPU box): smoke, GPU tests, default bench (with CPU baseline),
# kernel-trace + PMC profile of the same command.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-art}
mkdir -p $OUT
timeout -k 10 300 python3 __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke-fail > $OUT/done.txt; exit 1; }
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail > $OUT/done.txt; exit 1; }
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench-fail > $OUT/done.txt; exit 1; }
TAG=${TAG:-art}/prof bash tools/gpu/profile.sh || { echo prof-fail > $OUT/done.txt; exit 1; }
echo ok > $OUT/done.txt
