#!/bin/bash
# Round 6, second experiment call (GPU box, repo root): the 80-B quantized-node variant -- its
# GPU suite, C3 A/B against the product, one PMC pass each -- then the section counts of C2 and C3.
set -o pipefail
export TMPDIR=/tmp
VARIANT=qnode TAG=r06_exp2/qnode ROUNDS=3 bash tools/gpu/variant_ab.sh || exit 1
VARIANT=qnode TAG=r06_exp2/qnode_pmc bash tools/gpu/variant_pmc.sh || exit 1
TAG=r06_exp2/sec_c2 COUNT=1 BENCH_ARGS="--config C2" bash tools/gpu/exp.sh || exit 1
TAG=r06_exp2/sec_c3 COUNT=1 bash tools/gpu/exp.sh || exit 1
echo done
