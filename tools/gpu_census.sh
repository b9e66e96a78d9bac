#!/bin/bash
# Per-kernel instruction census of the bench (run via gpurun from the repo root):
# lists the box's counters, then one rocprofv3 --pmc pass per counter set below
# (only names the box lists; <= 8 SQ + GRBM per pass), each over a 2-step C2
# bench.  Raw CSVs under gpurun_out/census_<TAG>/; tools/census.py summarises.
# usage: tools/gpu_census.sh TAG [CONFIG] [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-x}; cfg=${2:-c2}; shift 2 2>/dev/null
out=gpurun_out/census_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
sets=(
 "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_ANY"
 "SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64"
 "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA"
 "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64"
)
i=0
for s in "${sets[@]}"; do
  i=$((i+1))
  keep=""
  for c in $s; do grep -qw "$c" $out/counters.txt && keep="$keep $c"; done
  echo "pass $i:$keep"
  [ -z "$keep" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $keep --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/p$i" -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
echo census_ok
