#!/bin/bash
# Is the C3 launch VALU-issue bound?  (1) the counter list of this box; (2) the issue-cost probe
# (tools/gpu/micro/valu_cost: SIMD-cycles per instruction class at 1-8 waves per SIMD); (3) the C3 launch's
# VALU instruction mix by class, one --pmc pass per group (only the counters the box lists).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_valu
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || echo "list-avail rc=$?" >> $OUT/notes.txt
timeout -k 10 300 tools/gpu/micro/valu_cost > $OUT/valu_cost.txt 2>&1 || { echo probe-fail; cat $OUT/valu_cost.txt; exit 1; }
cat $OUT/valu_cost.txt
pick() {  # the counters of "$@" that the box lists
  local out=""
  for c in "$@"; do grep -qw "$c" $OUT/list_avail.txt && out="$out $c"; done
  echo $out
}
i=0
while read -r group; do
  i=$((i+1))
  cs=$(pick $group)
  echo "pass $i: $cs" | tee -a $OUT/passes.txt
  [ -z "$cs" ] && continue
  timeout -k 10 300 rocprofv3 --pmc $cs --kernel-trace --output-format csv -d $OUT/pmc_$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --one-stream > $OUT/pmc_$i.json 2> $OUT/pmc_$i.err \
      || { echo "pmc-fail $i"; tail -5 $OUT/pmc_$i.err; exit 1; }
done <<'EOF'
SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64
SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F16 SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INSTS_VSKIPPED SQ_INSTS_LDS
EOF
echo done | tee $OUT/done.txt
