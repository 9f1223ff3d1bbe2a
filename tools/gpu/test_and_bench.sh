#!/bin/bash
# GPU tests + bench sweep (run on the GPU box from the repo root).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 300 python3 __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke failed" > $OUT/done.txt; exit 1; }
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed" > $OUT/done.txt; exit 1; }
for th in ${THRESHOLDS:-24}; do
  PT_WF_THRESHOLD=$th timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench_th$th.json 2> $OUT/bench_th$th.err || { echo "bench failed th=$th" > $OUT/done.txt; exit 1; }
done
echo "ok" > $OUT/done.txt
