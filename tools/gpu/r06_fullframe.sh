#!/bin/bash
# Round 6, final kernel: whole C2, C3 and C4 frames on the GPU against the CPU oracle on every pixel (16 host threads),
# bit for bit (tests/test_gpu_fullframe_oracle.py); progress per band of rows in gpurun_out/r06_fullframe/log.txt.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_fullframe
mkdir -p $OUT
rm -f $OUT/log.txt
PT_FULL_FRAME=C2,C3,C4 PT_FULL_FRAME_LOG=$OUT/log.txt timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_fullframe_oracle.py \
    -m gpu -v --timeout 1050 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo fullframe-fail; tail -30 $OUT/pytest.log; exit 1; }
tail -4 $OUT/pytest.log
grep config $OUT/log.txt
echo done
