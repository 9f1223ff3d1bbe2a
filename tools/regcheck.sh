#!/bin/bash
# Register budget check of the wavefront kernels (CPU only): compiles pt_render.hip for gfx950 with
# extra flags ($*) and prints VGPRs / scratch / spills per wavefront kernel instance.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${RC_OUT:-/tmp/rc}
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I$ROOT/include -fno-slp-vectorize "$@" \
  -x hip --offload-arch=gfx950 --cuda-device-only -S -o $OUT/k.s $ROOT/cudapathtracer_amd/csrc/hip/pt_render.hip \
  -Rpass-analysis=kernel-resource-usage 2> $OUT/ru.txt || { tail -20 $OUT/ru.txt; exit 1; }
python3 - $OUT/ru.txt <<'PY'
import re, sys
cur = None
for l in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1); continue
    if cur and ("wf" in cur):
        for key in ("VGPRs:", "ScratchSize", "VGPRs Spill", "Occupancy"):
            if key in l:
                print(cur[:60], l.split("remark:")[1].strip().split(" [")[0])
PY
