#!/bin/bash
# Round 6, VALU-issue experiments (2): the octant node array (-7 VALU per walk step: every node fetch of a step
# from one offset; with the leaf-sign keys) -- its GPU suite, then C3 alternated over base / leafkey / oct, one
# PMC pass each of oct (VALU, memory-side bytes), and C2 / integrator-1 checks of the oct library.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_exp4
mkdir -p $OUT
PT_LIB=variants/oct/libptamd.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_oct.log 2>&1 || { echo pytest-fail; tail -30 $OUT/pytest_oct.log; exit 1; }
tail -1 $OUT/pytest_oct.log
for r in 1 2 3; do
  for v in oct leafkey base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err \
        || { echo "bench-fail $v $r"; tail -5 $OUT/${v}_$r.err; exit 1; }
    echo "$v $r $(python3 -c "import json;d=json.load(open('$OUT/${v}_$r.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['node_fetches'], r['tri_tests'])")" | tee -a $OUT/summary.txt
  done
done
for pmc in "SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  for v in oct base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $OUT/pmc_${v}_$tag -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_${v}_$tag.json 2> $OUT/pmc_${v}_$tag.err \
        || { echo "pmc-fail $v $tag"; exit 1; }
  done
done
for cfg in C2; do
  for v in oct base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline > $OUT/${v}_$cfg.json 2> $OUT/${v}_$cfg.err \
        || { echo "bench-fail $v $cfg"; exit 1; }
    echo "$v $cfg $(python3 -c "import json;d=json.load(open('$OUT/${v}_$cfg.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
  done
done
echo done
