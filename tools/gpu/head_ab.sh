#!/bin/bash
# Integrator 1 on the wavefront kernel (GPU box, repo root): the GPU suite (-k TESTS, default all),
# then the C3 bench with --integrator 1 for each setting in SWEEP ("VAR=a,VAR2=b ..."; "-" = defaults).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-headab}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
      > $OUT/pytest_gpu.log 2>&1 || { echo pytest-fail > $OUT/done.txt; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
i=0
for kv in ${SWEEP:--}; do
  i=$((i+1))
  envs=""; [ "$kv" != "-" ] && envs=$(echo $kv | tr ',' ' ')
  env $envs timeout -k 10 300 python3 bench.py --integrator 1 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
      > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "bench failed: $kv" > $OUT/done.txt; exit 1; }
  echo "$kv $(python3 -c "
import json;d=json.load(open('$OUT/b_$i.json'));r=d['roofline'] or {}
print(d['value'], d['ms_per_step'], d['mrays_per_s_traced'], r.get('walk_simd_util'), r.get('walk_phase_frac'), r.get('shade_phases'), r.get('node_fetches'))")" | tee -a $OUT/summary.txt
done
echo ok > $OUT/done.txt
