#!/bin/bash
# Round 6, final kernel: whole-frame oracle parity beyond r06_fullframe -- FF (configs, e.g. C2H,C4H) and PART (k/n
# horizontal band); progress per band of rows in gpurun_out/r06_fullframe2/log.txt.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_fullframe2
mkdir -p $OUT
PT_FULL_FRAME=${FF:?} PT_FULL_FRAME_PART=${PART:-0/1} PT_FULL_FRAME_LOG=$OUT/log.txt timeout -k 10 1080 python3 -u -m pytest \
    tests/test_gpu_fullframe_oracle.py -m gpu -v --timeout 1050 --timeout-method thread > $OUT/pytest_${FF//,/_}_${PART//\//of}.log 2>&1 \
    || { echo fullframe-fail; tail -30 $OUT/pytest_${FF//,/_}_${PART//\//of}.log; exit 1; }
grep config $OUT/log.txt | tail -3
echo done
