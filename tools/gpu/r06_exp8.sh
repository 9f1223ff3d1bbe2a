#!/bin/bash
# Round 6, final kernel: (1) node-miss sensitivity -- 256-B node records (-DPT_NODE256: node footprint x2, one line per
# visit, the same walk instructions) against the product, with a parity check, C3 alternated and an L2 pass each;
# (2) the plain `bench.py --gpus 8` over gloo (eight rank processes started by bench.py, all on the one GPU), with the
# reduce and with the gather collective: the driver's N = 8 command but for RCCL.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_exp8
mkdir -p $OUT
PT_LIB=variants/node256/libptamd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_random_scenes.py tests/test_gpu_parity_sweep.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_node256.log 2>&1 || { echo pytest-fail; tail -20 $OUT/pytest_node256.log; exit 1; }
tail -1 $OUT/pytest_node256.log
for r in 1 2 3; do
  for v in node256 base; do
    lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
    PT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-count > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err \
        || { echo "bench-fail $v $r"; tail -5 $OUT/${v}_$r.err; exit 1; }
    echo "$v $r $(python3 -c "import json;d=json.load(open('$OUT/${v}_$r.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
  done
done
for v in node256 base; do
  lib=variants/$v/libptamd.so; [ $v = base ] && lib=""
  PT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_$v -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err \
      || { echo "pmc-fail $v"; exit 1; }
done
for coll in reduce gather; do
  PT_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline --collective $coll \
      > $OUT/plain_gpus8_gloo_$coll.json 2> $OUT/plain_gpus8_gloo_$coll.err || { echo "gpus8-fail $coll"; tail -20 $OUT/plain_gpus8_gloo_$coll.err; exit 1; }
  echo "plain --gpus 8 gloo $coll: $(python3 -c "import json;d=json.load(open('$OUT/plain_gpus8_gloo_$coll.json'));print(d['value'], d['n_gpus'], d['image_finite'], d['config'].get('rank_launcher'), d['config'].get('collective'))")"
done
echo done
