set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?" >> gpurun_out/smoke.log
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --spp 16 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1; echo "bench rc=$?" >> gpurun_out/bench_small.log
tail -3 gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/bench_small.log
