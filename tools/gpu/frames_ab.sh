#!/bin/bash
# Frame loop A/B (GPU box, repo root): the GPU suite (-k TESTS, default all; NOTEST=1 skips it), then for the
# full frame and the 1/8 shard (SHARDS, default "1 8") the bench with the default frame loop (two streams for
# shards only), on one stream, on two streams, and blocking.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-frames}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
      > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for n in ${SHARDS:-1 8}; do
  steps=$(( ${STEPS:-6} * (n > 1 ? n / 2 : 1) ))
  for mode in "" "--one-stream" "--two-streams" "--sync-frames"; do
    tag=s${n}${mode:-_default}
    timeout -k 10 300 python3 bench.py --steps $steps --warmup 2 --no-cpu-baseline --no-count --sim-shards $n $mode ${BENCH_ARGS} \
        > $OUT/$tag.json 2> $OUT/$tag.err || { echo "fail $tag" > $OUT/done.txt; exit 1; }
    echo "$tag $(python3 -c "import json;d=json.load(open('$OUT/$tag.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
  done
done
echo ok > $OUT/done.txt
