#!/bin/bash
# Round 6: the block ray pool's rate (kPool) against the product, C3, counting pass included (walk_simd_util).
set -o pipefail
export TMPDIR=/tmp
TAG=r06_pool/perf ROUNDS=${ROUNDS:-2} NOCOUNT=" " CONFIGS="pool:PT_WF_POOL=1 prod: pool4:PT_WF_POOL=1,PT_WF_POOL_MIN=4 pool16:PT_WF_POOL=1,PT_WF_POOL_MIN=16" bash tools/gpu/ab.sh || exit 1
echo done
