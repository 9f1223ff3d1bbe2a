#!/bin/bash
# Round 6, first experiment call (GPU box, repo root): the GPU suite on the product (exhaustive trace for small
# scenes included), the C2 A/B of the exhaustive trace against the LDS walk, then the folded-child-word variant
# (VERDICT r05 item 2c): its suite, C3 A/B and one PMC pass each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_exp1
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo pytest-fail; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
TAG=r06_exp1/c2 ROUNDS=3 BENCH_ARGS="--config C2" NOCOUNT=" " \
  CONFIGS="brute: walk:PT_WF_BRUTE=0 brute3:PT_WF_BRUTE_ITERS=3 brute4:PT_WF_BRUTE_ITERS=4" bash tools/gpu/ab.sh || exit 1
VARIANT=fold TAG=r06_exp1/fold ROUNDS=3 bash tools/gpu/variant_ab.sh || exit 1
VARIANT=fold TAG=r06_exp1/fold_pmc bash tools/gpu/variant_pmc.sh || exit 1
echo done
