#!/bin/bash
# Round 6: the block ray pool (kPool, PT_WF_POOL=1) -- the GPU suite with the pool on (every
# integrator-0 render of a tree larger than the LDS top walks from it), then C3 A/B against the product.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_pool
mkdir -p $OUT
PT_WF_POOL=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${TESTS:+-k "$TESTS"} > $OUT/pytest_gpu_pool.log 2>&1 || { echo pytest-fail; tail -30 $OUT/pytest_gpu_pool.log; exit 1; }
tail -1 $OUT/pytest_gpu_pool.log
TAG=r06_pool/ab ROUNDS=${ROUNDS:-2} NOCOUNT=" " CONFIGS="pool:PT_WF_POOL=1 prod: ${EXTRA}" bash tools/gpu/ab.sh || exit 1
echo done
