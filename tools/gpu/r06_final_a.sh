#!/bin/bash
# Round-6 artifacts, part A (GPU box, repo root): smoke, the GPU suite, the default bench line (CPU baseline
# included) and the C3 profile (kernel trace + the PMC passes of tools/gpu/profile.sh).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_final}
mkdir -p $OUT
timeout -k 10 300 python3 __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke-fail > $OUT/done_a.txt; tail -20 $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo pytest-fail > $OUT/done_a.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench-fail > $OUT/done_a.txt; exit 1; }
echo "bench $(python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print(d['value'], d['ms_per_step'])")"
TAG=${TAG:-r06_final}/prof bash tools/gpu/profile.sh || { echo prof-fail > $OUT/done_a.txt; exit 1; }
# the kernel's own VALU streams replayed alone (tools/gpu/micro/walk_replay, generated from this kernel's ISA)
timeout -k 10 120 tools/gpu/micro/walk_replay > $OUT/walk_replay.txt 2>&1 || { echo replay-fail > $OUT/done_a.txt; exit 1; }
echo ok > $OUT/done_a.txt
