#!/bin/bash
# Round artifacts, part A (GPU box, repo root): smoke, the GPU suite, the default bench line (CPU baseline
# included) and the C3 profile (kernel trace of the bench's own frame loop + the PMC passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 300 python3 __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke-fail > $OUT/done.txt; exit 1; }
echo smoke ok
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo pytest-fail > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench-fail > $OUT/done.txt; exit 1; }
echo bench ok
TAG=${TAG:-final}/prof bash tools/gpu/profile.sh || { echo prof-fail > $OUT/done.txt; exit 1; }
echo ok > $OUT/done.txt
