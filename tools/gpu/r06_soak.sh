#!/bin/bash
# Round 6, final kernel: the C3 bench line ten times back to back at the driver's step count (20 timed frames each),
# for the run-to-run spread of `value` on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_soak
mkdir -p $OUT
for r in $(seq 10); do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$r.json 2> $OUT/bench_$r.err \
      || { echo "bench-fail $r"; tail -5 $OUT/bench_$r.err; exit 1; }
  echo "$r $(python3 -c "import json;d=json.load(open('$OUT/bench_$r.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['bound'], (r.get('valu_issue') or {}).get('frac'))")" | tee -a $OUT/summary.txt
done
echo done
