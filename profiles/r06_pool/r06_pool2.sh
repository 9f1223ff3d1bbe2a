#!/bin/bash
# Round 6: pool mode, second build (walker-own rings, results validated by the slot word, waves wait for their own
# in-flight rays): bit-exactness on the debug frames and a subset of the GPU suite, then the C3 rate.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_pool2
MODES="PT_WF_POOL=1,PT_WF_POOL_SELF=8" timeout -k 10 300 python3 tools/gpu/pool_debug.py gpurun_out/r06_pool2/dbg > gpurun_out/r06_pool2/dbg.log 2>&1 || { tail -20 gpurun_out/r06_pool2/dbg.log; exit 1; }
grep -v "^   px" gpurun_out/r06_pool2/dbg.log
PT_WF_POOL=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/r06_pool2/pytest.log 2>&1; tail -3 gpurun_out/r06_pool2/pytest.log
TAG=r06_pool2/perf ROUNDS=1 NOCOUNT=" " CONFIGS="pool:PT_WF_POOL=1 prod: pool16:PT_WF_POOL=1,PT_WF_POOL_MIN=16" bash tools/gpu/ab.sh || exit 1
echo done
