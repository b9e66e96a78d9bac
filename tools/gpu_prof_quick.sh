#!/bin/bash
# Quick per-kernel profile of one bench configuration: kernel stats, then the
# HBM fetch and the SQ issue counters in separate passes (gpurun, repo root).
# usage: tools/gpu_prof_quick.sh TAG CONFIG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; cfg=$2; shift 2
out=gpurun_out/pq_$tag
mkdir -p $out
export TMPDIR=/tmp
pb="python3 bench.py --config $cfg --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/stats" -- $pb --steps 3 --warmup 1 "$@" > $out/stats.log 2>&1 || { echo stats_fail; tail -5 $out/stats.log; exit 1; }
tail -1 $out/stats.log | cut -c1-200
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/fetch" -- $pb --steps 1 --warmup 1 "$@" > $out/fetch.log 2>&1 || { echo fetch_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/sq" -- $pb --steps 1 --warmup 1 "$@" > $out/sq.log 2>&1 || { echo sq_fail; exit 1; }
echo pq_ok
