#!/bin/bash
# rocprofv3 counter passes over tools/pmc_probe.py (run via gpurun from the repo root).
# usage: tools/pmc_session.sh TAG [env assignments for the engine, e.g. DSCE_STAGE=fused]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
p=1
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F64"; do
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/p$p" -- python3 tools/pmc_probe.py > $out/p$p.log 2>&1 || { echo "pass $p failed"; tail -5 $out/p$p.log; exit 1; }
  p=$((p+1))
done
python3 tools/pmc_table.py $out > $out/table.txt && cat $out/table.txt
