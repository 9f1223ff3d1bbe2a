#!/bin/bash
# Per-GPU rate of one shard of N (bench.py --sim-shards N: shard 0 of N on this GPU; the whole-job
# rate at N GPUs is N x this), for each N in SHARDS (default "1 2 4 8": 1 = the full frame, the
# reference for the ratios), on the GPU box from the repo root.  BENCH_ARGS passes e.g. --sync-frames.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shardsim}
mkdir -p $OUT
for n in ${SHARDS:-1 2 4 8}; do
  steps=$(( ${STEPS:-4} * (n > 1 ? n / 2 : 1) ))
  timeout -k 10 300 python3 bench.py --steps $steps --warmup 2 --no-cpu-baseline --no-count --sim-shards $n ${BENCH_ARGS} \
      > $OUT/s_$n.json 2> $OUT/s_$n.err || { echo "fail $n" > $OUT/done.txt; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$OUT/s_$n.json'));print(d['value'], d['ms_per_step'], d['roofline'])")" >> $OUT/summary.txt
done
python3 - "$OUT/summary.txt" >> $OUT/summary.txt <<'PY'
import sys
rows = [l.split()[:3] for l in open(sys.argv[1]) if l[0].isdigit()]
full = {int(n): float(v) for n, v, _ in rows}
if 1 in full:
    for n in sorted(full):
        print("shards %d per-GPU %.1f Msamples/s = %.1f%% of the full frame -> projected %d-GPU job %.2fx"
              % (n, full[n], 100 * full[n] / full[1], n, n * full[n] / full[1]))
PY
echo ok > $OUT/done.txt
