#!/bin/bash
# Round 6, VALU-issue experiments: the leaf-sign stack keys (-DPT_LEAF_SIGN_KEYS: 3 fewer VALU per walk step,
# predicted +0.8-1.0% at C3 if the launch is VALU-issue bound) -- its GPU suite, a C3 A/B against the
# in-tree library (alternated), and one PMC pass each for the VALU count.
set -o pipefail
export TMPDIR=/tmp
VARIANT=leafkey TAG=r06_exp3/leafkey ROUNDS=3 bash tools/gpu/variant_ab.sh || exit 1
VARIANT=leafkey TAG=r06_exp3/leafkey_pmc PMC="SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU" bash tools/gpu/variant_pmc.sh || exit 1
echo done
