#!/bin/bash
# Baseline profile of the render kernel (run on the GPU box from the repo root).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_ktrace.json 2> $OUT/bench_ktrace.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count > $OUT/bench_write.json 2> $OUT/bench_write.err && \
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $OUT/pmc_sq -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count > $OUT/bench_sq.json 2> $OUT/bench_sq.err && \
timeout -k 10 600 python3 bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err
echo "exit=$?" > $OUT/done.txt
