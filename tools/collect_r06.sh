#!/bin/bash
# Copy the round-6 final runs (gpurun_out/r06_final: tools/gpu/r06_final_{a,b1,b2}.sh) into profiles/r06_final*: kernel
# stats + PMC summaries per config (tools/summarize_profile.py), their profiles/traffic.json entries
# (tools/update_traffic.py; entries of other kernel hashes are dropped), the bench lines, shard simulations, host rates.
# PART=a|b1|b2 (default all that exist).
set -e
S=gpurun_out/r06_final
P=profiles/r06_final
py() { python3 tools/summarize_profile.py $1 $2 > /dev/null; python3 tools/update_traffic.py $2 "${@:3}" > /dev/null; }
if [ -d $S/prof ]; then
  py $S/prof $P
  cp $S/smoke.log $S/pytest_gpu.log $S/bench_default.json $P/
fi
if [ -d $S/configs ]; then
  py $S/configs/C2 ${P}_C2 1024 1024 64 8 0 1
  py $S/configs/C4 ${P}_C4 1920 1080 1024 3 0 1
  py $S/configs/C5 ${P}_C5 3840 2160 4096 16 0 1
  py $S/head/C3 ${P}_head 1920 1080 256 3 1 1
  for c in C2 C4 C5; do cp $S/configs/bench_$c.json ${P}_$c/bench.json; done
  cp $S/head/bench_C3.json ${P}_head/bench.json
fi
if [ -d $S/shard8 ]; then
  for n in 2 4 8; do py $S/shard$n/C3 ${P}_shard$n 1920 1080 256 3 0 $n; cp $S/shard$n/bench_C3.json ${P}_shard$n/bench.json; done
  for c in C3 C4; do mkdir -p $P/shardsim_$c; cp $S/shardsim_$c/*.json $S/shardsim_$c/summary.txt $P/shardsim_$c/; done
  cp $S/host_rate.json $S/plain_gpus2_gloo.json $P/
fi
python3 - <<'PY'
import json, bench
p = 'profiles/traffic.json'; d = json.load(open(p)); sha = bench.kernel_source_sha256()
d['entries'] = [e for e in d['entries'] if e['kernel_source_sha256'] == sha]
json.dump(d, open(p, 'w'), indent=1)
for e in d['entries']:
    print(e['profile'], e['config'], round(e['kernel_ms'], 2), round(e['traffic_bytes_per_launch'] / 1e9, 2), 'GB',
          (e.get('binding') or {}).get('limiter'))
PY
