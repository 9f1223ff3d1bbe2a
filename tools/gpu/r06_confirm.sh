#!/bin/bash
# Round 6, the final kernel (leaf-sign keys): the CF_CHUNK0 device check (-DPT_DEBUG_CHECKS) over the GPU suite and
# C3 shard frames; a 2000-case randomised parity sweep; the plain `bench.py --gpus 4` over gloo (four rank processes
# started by bench.py itself, all on the one GPU).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_confirm
mkdir -p $OUT
PT_LIB=variants/debugchecks/libptamd.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_debugchecks.log 2>&1 || { echo pytest-fail; tail -30 $OUT/pytest_debugchecks.log; exit 1; }
tail -1 $OUT/pytest_debugchecks.log
for n in 1 4 8; do
  PT_LIB=variants/debugchecks/libptamd.so timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count \
      --sim-shards $n > $OUT/dbg_shard_$n.json 2> $OUT/dbg_shard_$n.err || { echo "shard-fail $n"; tail -5 $OUT/dbg_shard_$n.err; exit 1; }
  echo "debug build, shard 0 of $n: $(python3 -c "import json;d=json.load(open('$OUT/dbg_shard_$n.json'));print(d['value'], d['image_finite'])")"
done
rm -f $OUT/sweep.jsonl
PT_PARITY_SWEEP=2000 PT_PARITY_SWEEP_LOG=$OUT/sweep.jsonl timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity_sweep.py \
    -m gpu -q --timeout 300 --timeout-method thread > $OUT/sweep.log 2>&1 || { echo sweep-fail; tail -30 $OUT/sweep.log; exit 1; }
tail -1 $OUT/sweep.log
PT_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/plain_gpus4_gloo.json \
    2> $OUT/plain_gpus4_gloo.err || { echo gpus4-fail; tail -20 $OUT/plain_gpus4_gloo.err; exit 1; }
echo "plain --gpus 4 (gloo): $(python3 -c "import json;d=json.load(open('$OUT/plain_gpus4_gloo.json'));print(d['value'], d['n_gpus'], d['image_finite'], d['config'].get('rank_launcher'))")"
echo done
