#!/bin/bash
# Round 6, final kernel: the wavefront knobs around their defaults (walk threshold 56, root-first visits 4, shading
# iterations 2) and the render BVH4's cost knobs (DP collapse triangle cost 0.3, binary SAH node cost 1), C3 alternated, 2 rounds.
TAG=r06_knobs ROUNDS=2 CONFIGS="def: thr52:PT_WF_THRESHOLD=52 thr60:PT_WF_THRESHOLD=60 rf3:PT_WF_ROOT_FIRST=3 rf5:PT_WF_ROOT_FIRST=5 it3:PT_WF_ITERS=3 ct02:PT_COLLAPSE_CT=0.2 ct05:PT_COLLAPSE_CT=0.5 lnc15:PT_LEAF_NODE_COST=1.5" \
  bash tools/gpu/ab.sh
