#!/bin/bash
# Counter passes over the bench command (run via gpurun from the repo root):
#   tools/gpu_pmc_bench.sh TAG [bench args...]
# kernel stats, FETCH_SIZE, WRITE_SIZE and one SQ pass (prof_summary.py SQ_COUNTERS),
# each its own rocprofv3 run; prints the per-kernel counter table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_stats" -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $out/stats.log 2>&1 || { echo stats_fail; tail -5 $out/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_fetch" -- $B > $out/fetch.log 2>&1 || { echo fetch_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_write" -- $B > $out/write.log 2>&1 || { echo write_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_sq" -- $B > $out/sq.log 2>&1 || { echo sq_fail; exit 1; }
python3 tools/pmc_table.py $out/prof_fetch $out/prof_write $out/prof_sq > $out/table.txt && cut -c1-250 $out/table.txt | grep -E "kernel|k_mic|k_pic|k_jakes|k_txrx|k_tx_sym"
tail -1 $out/stats.log | cut -c1-300
echo all_ok
