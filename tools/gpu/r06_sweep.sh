#!/bin/bash
# Randomised parity sweep on the product kernel: tests/test_gpu_parity_sweep.py with PT_PARITY_SWEEP cases (random
# soups x random image size / spp / depth / integrator / lens / camera / seed, plus random rays through pt_trace),
# each bit-exact against the oracle; one JSON line per case in the log.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_sweep
mkdir -p $OUT
rm -f $OUT/cases.jsonl
PT_PARITY_SWEEP=${N:-200} PT_PARITY_SWEEP_LOG=$OUT/cases.jsonl timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_parity_sweep.py \
    -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo sweep-fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo done
