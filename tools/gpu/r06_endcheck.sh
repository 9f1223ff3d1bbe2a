#!/bin/bash
# Round 6 end check on the committed tree (what the driver runs at round end): smoke, the whole GPU suite, the default
# bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_endcheck
mkdir -p $OUT
timeout -k 10 300 python3 __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke-fail; tail -20 $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo pytest-fail; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench-fail; tail -10 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['bound'], r['frac'], (r.get('valu_issue') or {}).get('frac'), d['cpu_baseline']['value'])"
echo done
